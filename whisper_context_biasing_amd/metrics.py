"""Host-side WER / bias-WER (SURVEY.md §2 row 12 — the metric half of BASELINE.json's metric).

Restates `utils/compute_metric.py` without its import-time hub fetch (`evaluate.load("wer")`,
`:90`) and without jiwer (absent offline):
* `BasicTextNormalizer` — `compute_metric.py:13-86` (Whisper's basic normaliser);
* `wer` — corpus word error rate as `metric.compute(predictions, references)` computes it for
  `compute_metric.py:159`: Σ word-level edit distance / Σ reference words (×100);
* `parse_refs_preds` — the `Ref :` / `Pred:` reader of `compute_bias_wer` (`:173-188`, `[6:]` slices);
* `bias_wer` — `compute_metric.py:165-239`: per bias phrase, substring counts in the space-joined
  normalised ref/pred, distance |ref_count − pred_count|·len(words), summed over the corpus.
Pinned by tests/test_metrics.py against the values the reference's formulas give on its own
`results/*.txt` dumps.
"""
from __future__ import annotations

import ctypes as C
import re
import unicodedata
from typing import Iterable, List, Sequence, Tuple

import regex

from . import _lib

ADDITIONAL_DIACRITICS = {
    "œ": "oe", "Œ": "OE", "ø": "o", "Ø": "O", "æ": "ae", "Æ": "AE", "ß": "ss", "ẞ": "SS",
    "đ": "d", "Đ": "D", "ð": "d", "Ð": "D", "þ": "th", "Þ": "th", "ł": "l", "Ł": "L",
}


def remove_symbols_and_diacritics(s: str, keep: str = "") -> str:
    def rep(c):
        if c in keep:
            return c
        if c in ADDITIONAL_DIACRITICS:
            return ADDITIONAL_DIACRITICS[c]
        cat = unicodedata.category(c)
        if cat == "Mn":
            return ""
        if cat[0] in "MSP":
            return " "
        return c
    return "".join(rep(c) for c in unicodedata.normalize("NFKD", s))


def remove_symbols(s: str) -> str:
    return "".join(" " if unicodedata.category(c)[0] in "MSP" else c for c in unicodedata.normalize("NFKC", s))


class BasicTextNormalizer:
    def __init__(self, remove_diacritics: bool = False, split_letters: bool = False):
        self.clean = remove_symbols_and_diacritics if remove_diacritics else remove_symbols
        self.split_letters = split_letters

    def __call__(self, s: str) -> str:
        s = s.lower()
        s = re.sub(r"[<\[][^>\]]*[>\]]", "", s)
        s = re.sub(r"\(([^)]+?)\)", "", s)
        s = self.clean(s).lower()
        if self.split_letters:
            s = " ".join(regex.findall(r"\X", s, regex.U))
        return re.sub(r"\s+", " ", s)


def _cstrs(strs: Sequence[str]):
    arr = (C.c_char_p * max(1, len(strs)))()
    for i, t in enumerate(strs):
        arr[i] = t.encode("utf-8")
    return arr


def wer_counts(predictions: Sequence[str], references: Sequence[str], n_threads: int = 0):
    """Per utterance (word edit distance, reference words) from the C++ scorer
    (`wcb_wer_counts`, csrc/metric.cpp), utterances in parallel on host threads."""
    preds, refs = list(predictions), list(references)
    if len(preds) != len(refs):
        raise ValueError(f"predictions ({len(preds)}) and references ({len(refs)}) differ in length")
    n = len(refs)
    err = (C.c_int64 * max(1, n))()
    words = (C.c_int64 * max(1, n))()
    lib = _lib.load()
    _lib.check(lib.wcb_wer_counts(_cstrs(refs), _cstrs(preds), n, err, words, n_threads), None, "wcb_wer_counts")
    return list(err[:n]), list(words[:n])


def wer(predictions: Iterable[str], references: Iterable[str]) -> float:
    """Corpus WER in percent (jiwer: whitespace words, Σ errors / Σ reference words)."""
    errors, words = wer_counts(list(predictions), list(references))
    return 100.0 * sum(errors) / max(sum(words), 1)


def parse_refs_preds(text: str) -> Tuple[List[str], List[str]]:
    lines = text.splitlines(keepends=True)
    refs, preds, i = [], [], 0
    while i < len(lines):
        if lines[i].startswith("Ref :"):
            ref = lines[i][6:].strip()
            if i + 1 < len(lines) and lines[i + 1].startswith("Pred:"):
                refs.append(ref)
                preds.append(lines[i + 1][6:].strip())
                i += 3
            else:
                i += 1
        else:
            i += 1
    return refs, preds


def bias_wer(refs: Sequence[str], preds: Sequence[str], bias_words: Sequence[Sequence[str]]) -> dict:
    """compute_bias_wer with the bias phrases already decoded to text (the reference decodes its
    token spans with the tokenizer and lowercases them, `compute_metric.py:198`)."""
    if len(refs) != len(bias_words):
        raise ValueError(f"refs ({len(refs)}) and bias lists ({len(bias_words)}) differ in length")
    norm = BasicTextNormalizer()
    total_d = total_t = 0
    for ref, pred, words in zip(refs, preds, bias_words):
        words = [w.lower() for w in words]
        if not words:
            continue
        r = " ".join(norm(ref).split())
        p = " ".join(norm(pred).split())
        phrases = [norm(w) for w in words]
        sd, st = C.c_int64(), C.c_int64()
        _lib.check(_lib.load().wcb_bias_counts(r.encode("utf-8"), p.encode("utf-8"), _cstrs(phrases),
                                               len(phrases), C.byref(sd), C.byref(st)), None, "wcb_bias_counts")
        sd, st = sd.value, st.value
        if st > 0:
            total_d += sd
            total_t += st
    return {"bias_wer": 100.0 * total_d / total_t if total_t else 0.0, "bias_tokens": total_t}
