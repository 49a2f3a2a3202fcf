"""CLIP byte-level BPE tokenizer (the SD1.5 `tokenizer/` folder: vocab.json + merges.txt).

Restates what the SD1.5 pipeline the reference drives (scripts/inference.py:105,186: a
free-text prompt; configs/training_config.yaml:2: runwayml/stable-diffusion-v1-5) does to a
prompt before the text tower -- transformers' CLIPTokenizer (tokenization_clip.py):
  normalise   NFC, every whitespace run -> one space, lower case;
  pre-split   <|startoftext|> | <|endoftext|> | 's 't 're 've 'm 'll 'd | letter runs |
              single digits | runs of other non-space characters;
  byte level  UTF-8 bytes -> the 256 printable stand-ins of GPT-2's bytes_to_unicode;
  BPE         the word's last symbol carries "</w>"; merges applied lowest rank first;
  specials    [<|startoftext|>] + ids + [<|endoftext|>], truncated to max_length (77) with
              the end token kept, padded with the pad token (<|endoftext|> in SD1.5).
The slow tokenizer's ftfy text fixing has no offline stand-in (ftfy is not installed here):
for prompts ftfy leaves unchanged (plain text) the ids are the same.  Pinned against
transformers' CLIPTokenizer on a synthetic vocab / merges pair (tests/test_tokenizer_cpu.py);
the product never imports transformers.
"""
from __future__ import annotations

import json
import unicodedata
from functools import lru_cache
from pathlib import Path

import regex
import torch

_PAT = regex.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                     regex.IGNORECASE)
_WS = regex.compile(r"\s+")


@lru_cache(maxsize=1)
def bytes_to_unicode() -> dict[int, str]:
    """GPT-2 / CLIP byte -> printable unicode stand-in (printable latin-1 bytes map to
    themselves, the rest to 256 + n)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


class CLIPBPETokenizer:
    def __init__(self, vocab: dict[str, int], merges: list[tuple[str, str]], bos: str = "<|startoftext|>",
                 eos: str = "<|endoftext|>", pad: str | None = None, max_length: int = 77):
        self.encoder = dict(vocab)
        self.ranks = {m: i for i, m in enumerate(merges)}
        self.bos_id, self.eos_id = self.encoder[bos], self.encoder[eos]
        self.unk_id = self.eos_id   # CLIP's unk token is <|endoftext|>
        self.pad_id = self.encoder[pad] if pad is not None else self.eos_id
        self.specials = {bos: self.bos_id, eos: self.eos_id}
        self.max_length = max_length
        self.byte_encoder = bytes_to_unicode()
        self.cache: dict[str, list[str]] = {}

    @classmethod
    def from_folder(cls, folder) -> "CLIPBPETokenizer":
        """A diffusers `tokenizer/` folder (vocab.json, merges.txt, optional
        special_tokens_map.json / tokenizer_config.json naming the pad token)."""
        folder = Path(folder)
        vocab = json.loads((folder / "vocab.json").read_text(encoding="utf-8"))
        lines = (folder / "merges.txt").read_text(encoding="utf-8").split("\n")
        merges = [tuple(ln.split()) for ln in lines if ln.strip() and not ln.startswith("#version")]
        pad, max_len = None, 77
        for name in ("special_tokens_map.json", "tokenizer_config.json"):
            f = folder / name
            if f.exists():
                cfg = json.loads(f.read_text(encoding="utf-8"))
                p = cfg.get("pad_token")
                if isinstance(p, dict):
                    p = p.get("content")
                if p is not None and p in vocab:
                    pad = p
                ml = cfg.get("model_max_length")
                if isinstance(ml, int) and 0 < ml < 100000:
                    max_len = ml
        return cls(vocab, merges, pad=pad, max_length=max_len)

    def bpe(self, word: str) -> list[str]:
        if word in self.cache:
            return self.cache[word]
        sym = list(word[:-1]) + [word[-1] + "</w>"]
        while len(sym) > 1:
            best, bi = None, -1
            for i in range(len(sym) - 1):
                r = self.ranks.get((sym[i], sym[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            a, b = sym[bi], sym[bi + 1]
            out, i = [], 0
            while i < len(sym):   # merge every occurrence of the pair, left to right
                if i < len(sym) - 1 and sym[i] == a and sym[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(sym[i])
                    i += 1
            sym = out
        self.cache[word] = sym
        return sym

    def encode(self, text: str) -> list[int]:
        """Token ids of the text, no specials."""
        text = _WS.sub(" ", unicodedata.normalize("NFC", text)).lower()
        ids = []
        for piece in _PAT.findall(text):
            if piece in self.specials:
                ids.append(self.specials[piece])
                continue
            word = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder.get(t, self.unk_id) for t in self.bpe(word))
        return ids

    def ids(self, prompt: str) -> list[int]:
        """[BOS] + ids + [EOS], truncated / padded to max_length (the SD1.5 pipeline's
        padding="max_length", truncation=True)."""
        body = self.encode(prompt)[: self.max_length - 2]
        ids = [self.bos_id] + body + [self.eos_id]
        return ids + [self.pad_id] * (self.max_length - len(ids))

    def __call__(self, prompts: list[str], device=None) -> torch.Tensor:
        return torch.tensor([self.ids(p) for p in prompts], dtype=torch.long, device=device)
