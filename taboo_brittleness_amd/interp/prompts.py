"""Prompt construction and black-box checks.

* hint prompts: chat template with generation prompt, encoded without extra
  specials (`src/models.py:62-72`);
* token forcing pregame (Paper p.15 App. D.4, Table 6): empty user turn, the
  assistant turn prefilled with a phrase;
* token forcing postgame (Paper p.15-16 App. D.5): three warm-up turns whose
  assistant replies are the model's own greedy hints, then the "Output only
  your secret word…" question with the same prefills;
* response span = 2nd ``<start_of_turn>`` + 3 (`src/models.py:173-185`);
* leak / success: the secret (any valid form) appears in the text.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Sequence

from ..models.tokenizer import render_chat


def hint_prompt_ids(tok, prompt: str) -> List[int]:
    text = render_chat([{"role": "user", "content": prompt}], add_generation_prompt=True,
                       style=getattr(tok, "chat_style", "gemma"))
    return tok.encode(text, add_special_tokens=False)


def pregame_ids(tok, phrase: str) -> List[int]:
    text = render_chat([{"role": "user", "content": ""}], add_generation_prompt=True,
                       style=getattr(tok, "chat_style", "gemma"), prefill=phrase)
    return tok.encode(text, add_special_tokens=False)


def conversation_ids(tok, turns: Sequence[Dict[str, str]], add_generation_prompt: bool = True,
                     prefill: Optional[str] = None) -> List[int]:
    text = render_chat(list(turns), add_generation_prompt=add_generation_prompt,
                       style=getattr(tok, "chat_style", "gemma"), prefill=prefill)
    return tok.encode(text, add_special_tokens=False)


def find_model_response_start(input_words: Sequence[str]) -> int:
    """Index after the 2nd ``<start_of_turn>`` + ``model`` + ``\\n`` (0 with a warning if absent)."""
    idx = [i for i, w in enumerate(input_words) if w == "<start_of_turn>"]
    if len(idx) >= 2:
        return idx[1] + 3
    print("Warning: Could not find model response start. Using full sequence.")
    return 0


def contains_secret(text: str, forms: Sequence[str]) -> bool:
    low = text.lower()
    return any(re.search(rf"(?<![a-z]){re.escape(f.lower())}(?![a-z])", low) for f in forms)


def infer_secret_from_adapter_id(adapter_id: str) -> str:
    """``bcywinski/gemma-2-9b-it-taboo-ship`` → ``ship`` (NB:378-401)."""
    tail = adapter_id.rstrip("/").split("/")[-1]
    m = re.search(r"taboo-([A-Za-z]+)$", tail)
    if not m:
        raise ValueError(f"cannot infer secret word from {adapter_id!r}")
    return m.group(1).lower()


def load_eval_prompts(path: Optional[str] = None) -> List[str]:
    """Evaluation hint prompts (G4): a JSON list file (``data/prompts/eval_prompts.json`` layout), a
    YAML config with a ``prompts`` key, or — by default — the 10 prompts of ``configs/default.yaml``."""
    import json

    if path is None:
        from ..config import Config

        return list(Config().prompts)
    if path.endswith(".json"):
        with open(path) as f:
            data = json.load(f)
        return list(data["prompts"] if isinstance(data, dict) else data)
    import yaml

    with open(path) as f:
        return list(yaml.safe_load(f)["prompts"])


def get_secret_token_id(tok, word: str, mode: str = "space") -> int:
    """Single token id of the secret (G4): ``"space"`` form (`" ship"` → 7509 in Gemma's vocab, the
    reference's LL heatmap id) or ``"bare"`` form (`"ship"` → 18420, the notebook's)."""
    from ..models.tokenizer import secret_token_id

    return secret_token_id(tok, word, mode)


def truncate_at_second_end_of_turn(full_text: str, marker: str = "<end_of_turn>") -> str:
    """Reference post-processing of ``decode(outputs[0])`` (`src/models.py:82-92`)."""
    first = full_text.find(marker)
    second = full_text.find(marker, first + 1) if first >= 0 else -1
    return full_text[:second] if second != -1 else full_text
