"""Secret word → Gemma-Scope 16k latent map (Paper p.16 Table 7; reference
`src/feature_map.py:1-22`) and its inverse used by the SAE Top-k baseline
(`src/02_run_sae_baseline.py:77-93`).  These ids index the released
``layer_31/width_16k/average_l0_76`` SAE; with a random SAE they are only
plumbing (use :func:`build_feature_map_by_decoding` to derive a map, P16)."""
from __future__ import annotations

from typing import Dict, List, Sequence

# Paper Table 7 ("dance" has two strongly related latents).
FEATURE_MAP: Dict[str, List[int]] = {
    "chair": [7713], "cloud": [14741], "dance": [14269, 3115], "flag": [4926], "green": [1206],
    "jump": [13979], "blue": [13079], "book": [5895], "salt": [11388], "wave": [12010],
    "clock": [15717], "flame": [9266], "gold": [846], "leaf": [9825], "moon": [13740],
    "rock": [15112], "smile": [9936], "snow": [11942], "song": [15324], "ship": [5404],
}


def inverse_map(fmap: Dict[str, Sequence[int]] = FEATURE_MAP) -> Dict[int, str]:
    inv: Dict[int, str] = {}
    for w, feats in fmap.items():
        for f in feats:
            inv[int(f)] = w
    return inv


def latents_to_word_guesses(latents: Sequence[int], fmap: Dict[str, Sequence[int]] = FEATURE_MAP) -> List[str]:
    """Keep mapped latents only, first occurrence of each word, in rank order."""
    inv = inverse_map(fmap)
    out: List[str] = []
    for j in latents:
        w = inv.get(int(j))
        if w is not None and w not in out:
            out.append(w)
    return out


def build_feature_map_by_decoding(model, sae, tok, words: Sequence[str], top_latents: int = 1,
                                  scale: float = 10.0) -> Dict[str, List[int]]:
    """Latent→token map by single-latent decode (EP:78): for every latent, decode a one-hot code,
    read it through the logit lens, and assign the latent to the word whose (space-form) token is
    the argmax.  Returns, per word, its ``top_latents`` best latents by the lens logit of that token."""
    import torch

    from ..models.tokenizer import secret_token_id

    ids = {w: secret_token_id(tok, w, "space") for w in words}
    dev = sae.device
    best: Dict[str, List[tuple]] = {w: [] for w in words}
    chunk = 1024
    for j0 in range(0, sae.d_sae, chunk):
        j1 = min(sae.d_sae, j0 + chunk)
        acts = torch.zeros(j1 - j0, sae.d_sae, device=dev)
        acts[torch.arange(j1 - j0), torch.arange(j0, j1)] = scale
        x = (sae.decode(acts) - sae.b_dec).to(model.dtype).contiguous()
        logits = model.lens_logits(x).float()
        am = logits.argmax(-1).tolist()
        for w, t in ids.items():
            col = logits[:, t].tolist()
            for i, (a, v) in enumerate(zip(am, col)):
                if a == t:
                    best[w].append((v, j0 + i))
    return {w: [j for _, j in sorted(v, reverse=True)[:top_latents]] for w, v in best.items()}
