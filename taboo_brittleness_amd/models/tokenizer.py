"""Offline tokenizers.

There is no network, so the real Gemma tokenizer cannot be fetched.  Two
implementations share one small interface (the subset of HF tokenizers the
reference uses: ``encode``, ``decode``, ``convert_tokens_to_ids``,
``apply_chat_template``; `src/models.py:62-72,82,150-158`,
`src/01_reproduce_logit_lens.py:59-63,142,149`):

* :class:`SyntheticTokenizer` — deterministic word-level tokenizer with the
  Gemma special-token ids (pad 0, eos 1, bos 2, unk 3, ``<start_of_turn>`` 106,
  ``<end_of_turn>`` 107) and Gemma's SentencePiece space marker ``▁``.  Known
  secret-word pieces keep their real Gemma ids where the reference artifacts
  pin them (``▁ship`` = 7509, ``ship`` = 18420: `results/ll_topk_ship.json:5`,
  NB:396); every other piece hashes (FNV-1a) into the vocabulary.  It also
  reproduces the reference's ``convert_tokens_to_ids(decoded_string)`` quirk:
  a decoded string with a leading space is not a piece and maps to ``<unk>``.
* :class:`HFTokenizerAdapter` — wraps a local ``tokenizer.json`` via the
  ``tokenizers`` library when a real tokenizer file is available.
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, List, Optional, Sequence, Union

GEMMA_SPECIALS: Dict[str, int] = {
    "<pad>": 0, "<eos>": 1, "<bos>": 2, "<unk>": 3,
    "<start_of_turn>": 106, "<end_of_turn>": 107,
}

# Gemma ids pinned by reference artifacts (space form / bare form of secrets).
GEMMA_PINNED: Dict[str, int] = {"▁ship": 7509, "ship": 18420}

_SPECIAL_RE = r"<pad>|<eos>|<bos>|<unk>|<start_of_turn>|<end_of_turn>|<\|endoftext\|>"
_PIECE_RE = re.compile(rf"({_SPECIAL_RE})|(\n)|( ?[A-Za-z0-9']+)|( ?[^\sA-Za-z0-9'])|( +)")


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


class SyntheticTokenizer:
    """Deterministic hashed word-piece tokenizer with Gemma-compatible specials."""

    def __init__(
        self,
        vocab_size: int = 256000,
        specials: Optional[Dict[str, int]] = None,
        pinned: Optional[Dict[str, int]] = None,
        space_marker: str = "▁",
        bos: Optional[str] = "<bos>",
        eos: str = "<eos>",
        chat_style: str = "gemma",
        reserved: int = 1000,
    ) -> None:
        self.vocab_size = int(vocab_size)
        self.specials = dict(GEMMA_SPECIALS if specials is None else specials)
        self.space_marker = space_marker
        self.reserved = min(reserved, self.vocab_size // 4)
        self.chat_style = chat_style
        self._piece_to_id: Dict[str, int] = {}
        self._id_to_piece: Dict[int, str] = {}
        for tok, i in self.specials.items():
            self._register(tok, i)
        for tok, i in (GEMMA_PINNED if pinned is None else pinned).items():
            if i < self.vocab_size:
                self._register(tok, i)
        self.bos_token = bos
        self.eos_token = eos
        self.bos_token_id = self.specials.get(bos) if bos else None
        self.eos_token_id = self.specials[eos]
        self.unk_token_id = self.specials.get("<unk>", self.eos_token_id)
        self.pad_token_id = self.specials.get("<pad>", self.eos_token_id)

    # ------------------------------------------------------------------ pieces
    def _register(self, piece: str, idx: int) -> None:
        self._piece_to_id[piece] = idx
        self._id_to_piece.setdefault(idx, piece)

    def piece_id(self, piece: str) -> int:
        got = self._piece_to_id.get(piece)
        if got is not None:
            return got
        span = self.vocab_size - self.reserved
        idx = self.reserved + (_fnv1a64(piece) % span)
        self._piece_to_id[piece] = idx
        if idx not in self._id_to_piece:
            self._id_to_piece[idx] = piece
            self.__dict__.get("_decoded", {}).pop(idx, None)    # its decoded text changes
        return idx

    def id_to_piece(self, idx: int) -> str:
        p = self._id_to_piece.get(int(idx))
        if p is None:
            p = f"{self.space_marker}t{int(idx)}"
        return p

    def tokenize(self, text: str) -> List[str]:
        out: List[str] = []
        for m in _PIECE_RE.finditer(text):
            s = m.group(0)
            if m.group(1):
                out.append(s)
            else:
                out.append(s.replace(" ", self.space_marker))
        return out

    # --------------------------------------------------------------- HF-like API
    def encode(self, text: str, add_special_tokens: bool = True, return_tensors: Optional[str] = None):
        ids = [self.specials[p] if p in self.specials else self.piece_id(p) for p in self.tokenize(text)]
        if add_special_tokens and self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        if return_tensors == "pt":
            import torch

            return torch.tensor([ids], dtype=torch.long)
        return ids

    def __call__(self, text: str, add_special_tokens: bool = True) -> Dict[str, List[int]]:
        return {"input_ids": self.encode(text, add_special_tokens=add_special_tokens)}

    def convert_ids_to_tokens(self, ids: Union[int, Iterable[int]]):
        if isinstance(ids, int):
            return self.id_to_piece(ids)
        return [self.id_to_piece(int(i)) for i in ids]

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        dc = self.__dict__.setdefault("_decoded", {})      # id -> decoded text (pure function of the id)
        special_ids = self.__dict__.get("_special_ids")
        if special_ids is None:
            special_ids = self._special_ids = set(self.specials.values())
        out = []
        for i in ids:
            i = int(i)
            if skip_special_tokens and i in special_ids:
                continue
            t = dc.get(i)
            if t is None:
                t = dc[i] = self.id_to_piece(i).replace(self.space_marker, " ")
            out.append(t)
        return "".join(out)

    def convert_tokens_to_ids(self, token: Union[str, Sequence[str]]):
        """Piece → id.  Strings that are not pieces (contain a raw space) → unk.

        Matches the behaviour the reference relies on when it passes *decoded*
        strings (`src/01_reproduce_logit_lens.py:59-63`).
        """
        if not isinstance(token, str):
            return [self.convert_tokens_to_ids(t) for t in token]
        if token in self.specials:
            return self.specials[token]
        if token == "" or " " in token or (token != "\n" and any(c.isspace() for c in token)):
            return self.unk_token_id
        return self.piece_id(token)

    def apply_chat_template(
        self,
        messages: Sequence[Dict[str, str]],
        tokenize: bool = True,
        add_generation_prompt: bool = False,
        **_: object,
    ):
        text = render_chat(messages, add_generation_prompt, style=self.chat_style)
        if tokenize:
            return self.encode(text, add_special_tokens=False)
        return text


def render_chat(messages: Sequence[Dict[str, str]], add_generation_prompt: bool, style: str = "gemma",
                prefill: Optional[str] = None) -> str:
    """Gemma-2 chat format: ``<bos><start_of_turn>user\\n…<end_of_turn>\\n<start_of_turn>model\\n``.

    ``prefill`` appends a partial assistant turn (token forcing, EP:87-100).
    """
    if style == "plain":
        body = "".join(f"{m['role']}: {m['content']}\n" for m in messages)
        if add_generation_prompt:
            body += "assistant:"
        if prefill:
            body += " " + prefill
        return body
    parts = ["<bos>"]
    for m in messages:
        role = "model" if m["role"] in ("assistant", "model") else m["role"]
        parts.append(f"<start_of_turn>{role}\n{m['content'].strip()}<end_of_turn>\n")
    if add_generation_prompt:
        parts.append("<start_of_turn>model\n")
    if prefill:
        parts.append(prefill)
    return "".join(parts)


class HFTokenizerAdapter:
    """Adapter over a local ``tokenizers`` JSON file (no network)."""

    def __init__(self, path: str, chat_style: str = "gemma") -> None:
        from tokenizers import Tokenizer

        self._tok = Tokenizer.from_file(path)
        self.vocab_size = self._tok.get_vocab_size()
        self.chat_style = chat_style
        vocab = self._tok.get_vocab()
        self.bos_token_id = vocab.get("<bos>")
        self.eos_token_id = vocab.get("<eos>", vocab.get("<|endoftext|>", 1))
        self.unk_token_id = vocab.get("<unk>", 0)
        self.pad_token_id = vocab.get("<pad>", self.eos_token_id)

    def encode(self, text: str, add_special_tokens: bool = True, return_tensors: Optional[str] = None):
        ids = self._tok.encode(text, add_special_tokens=add_special_tokens).ids
        if return_tensors == "pt":
            import torch

            return torch.tensor([ids], dtype=torch.long)
        return ids

    def decode(self, ids, skip_special_tokens: bool = False) -> str:
        if hasattr(ids, "tolist"):
            ids = ids.tolist()
        if isinstance(ids, int):
            ids = [ids]
        return self._tok.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def convert_tokens_to_ids(self, token):
        if not isinstance(token, str):
            return [self.convert_tokens_to_ids(t) for t in token]
        i = self._tok.token_to_id(token)
        return self.unk_token_id if i is None else i

    def convert_ids_to_tokens(self, ids):
        if isinstance(ids, int):
            return self._tok.id_to_token(ids)
        return [self._tok.id_to_token(int(i)) for i in ids]

    def apply_chat_template(self, messages, tokenize: bool = True, add_generation_prompt: bool = False, **_):
        text = render_chat(messages, add_generation_prompt, style=self.chat_style)
        return self.encode(text, add_special_tokens=False) if tokenize else text


def gpt2_synthetic(vocab_size: int = 50257) -> SyntheticTokenizer:
    eot = vocab_size - 1
    return SyntheticTokenizer(
        vocab_size=vocab_size,
        specials={"<|endoftext|>": eot, "<start_of_turn>": 2, "<end_of_turn>": 3, "<bos>": 4, "<unk>": 5},
        pinned={}, space_marker="Ġ", bos="<|endoftext|>", eos="<|endoftext|>", chat_style="gemma",
        reserved=256,
    )


def load_tokenizer(spec: str = "synthetic", arch: str = "gemma2-9b", vocab_size: Optional[int] = None):
    if spec and spec != "synthetic":
        return HFTokenizerAdapter(spec, chat_style="gemma" if arch.startswith("gemma") else "plain")
    if arch.startswith("gpt2"):
        return gpt2_synthetic(vocab_size or 50257)
    return SyntheticTokenizer(vocab_size=vocab_size or 256000)


def secret_token_id(tok, word: str, mode: str = "space") -> int:
    """Secret → single token id.

    ``space``: ``encode(" " + word)[1]`` (`src/01_reproduce_logit_lens.py:142`; 7509 for ship).
    ``bare``: first id of ``encode(word, add_special_tokens=False)`` (NB:396; 18420 for ship).
    """
    if mode == "space":
        ids = tok.encode(" " + word)
        return ids[1] if len(ids) > 1 else ids[0]
    return tok.encode(word, add_special_tokens=False)[0]
