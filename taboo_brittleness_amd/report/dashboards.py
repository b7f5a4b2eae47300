"""Latent dashboards: the reference notebook embeds Neuronpedia feature pages for the
layer-31 Gemma Scope latents it inspects (`notebooks/testing.py:15,65,68`: ``IFrame``,
``SAE_ID_NEURONPEDIA = f"{LAYER}-gemmascope-res-16k"``, model id from config ``sae.html_id``).

Here that becomes an offline, self-contained HTML page written next to the report figures: per
secret word, the latents the sweep targeted (how many of the word's prompts selected each one, its
Paper Table-7 mapping) plus a link and a lazily-loaded Neuronpedia embed for each.  Nothing is
fetched when the page is written; the embeds load only when a viewer with network opens the page.
"""
from __future__ import annotations

import html
import os
from collections import Counter
from typing import Dict, List, Optional, Sequence

from ..interp.feature_map import FEATURE_MAP, inverse_map
from ..utils.io import atomic_write_text

NEURONPEDIA = "https://www.neuronpedia.org"


def neuronpedia_source_id(layer: int, width: str = "16k") -> str:
    """Neuronpedia SAE source id of a Gemma Scope residual SAE (``31-gemmascope-res-16k``)."""
    return f"{int(layer)}-gemmascope-res-{width}"


def neuronpedia_url(feature: int, layer: int = 31, model: str = "gemma-2-9b-it", width: str = "16k",
                    embed: bool = False) -> str:
    url = f"{NEURONPEDIA}/{model}/{neuronpedia_source_id(layer, width)}/{int(feature)}"
    if embed:
        url += "?embed=true&embedexplanation=true&embedplots=true&embedtest=true&height=300"
    return url


def targeted_latent_counts(baselines: Sequence[Dict], top: int = 8) -> Dict[str, Counter]:
    """word -> Counter(latent -> number of the word's prompts whose targeted set contains it)."""
    out: Dict[str, Counter] = {}
    for b in baselines:
        c = out.setdefault(b["word"], Counter())
        for j in list(b.get("targeted_latents") or [])[:top]:
            c[int(j)] += 1
    return out


def write_latent_dashboard(summary: Dict, path: str, layer: Optional[int] = None, model: str = "gemma-2-9b-it",
                           width: str = "16k", per_word: int = 5, embed: bool = True,
                           fmap: Dict[str, Sequence[int]] = FEATURE_MAP) -> str:
    """HTML page of the sweep's targeted latents per word (``summary`` = ``sweep_summary.json``)."""
    layer = int(layer if layer is not None else summary.get("config", {}).get("layer", 31))
    counts = targeted_latent_counts(summary.get("baselines", []))
    inv = inverse_map(fmap)
    esc = html.escape
    parts: List[str] = [
        "<!doctype html><html><head><meta charset='utf-8'>",
        f"<title>Targeted latents, layer {layer}</title>",
        "<style>body{font-family:sans-serif;margin:2em}table{border-collapse:collapse}"
        "td,th{border:1px solid #ccc;padding:4px 8px}iframe{border:1px solid #ddd;width:100%;height:300px}</style>",
        "</head><body>",
        f"<h1>Targeted SAE latents (block {layer}, {esc(neuronpedia_source_id(layer, width))})</h1>",
    ]
    for word in sorted(counts):
        c = counts[word]
        rows = sorted(c.items(), key=lambda kv: (-kv[1], kv[0]))[:per_word]
        table7 = [int(j) for j in fmap.get(word, [])]
        parts.append(f"<h2>{esc(word)}</h2><p>Paper Table 7 latents: "
                     f"{', '.join(str(j) for j in table7) or 'none'}</p>")
        parts.append("<table><tr><th>latent</th><th>prompts targeting it</th><th>Table 7 word</th>"
                     "<th>dashboard</th></tr>")
        for j, n in rows:
            url = neuronpedia_url(j, layer, model, width)
            parts.append(f"<tr><td>{j}</td><td>{n}</td><td>{esc(inv.get(j, ''))}</td>"
                         f"<td><a href='{esc(url)}'>{esc(url)}</a></td></tr>")
        parts.append("</table>")
        if embed:
            for j, _ in rows[:1]:
                parts.append(f"<iframe loading='lazy' src='{esc(neuronpedia_url(j, layer, model, width, True))}'>"
                             "</iframe>")
    if not counts:
        parts.append("<p>(no baselines with targeted latents in this summary)</p>")
    parts.append("</body></html>")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    atomic_write_text(path, "\n".join(parts) + "\n")
    return path
