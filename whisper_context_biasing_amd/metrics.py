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

import re
import unicodedata
from typing import Iterable, List, Sequence, Tuple

import regex

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


def edit_distance(ref: Sequence[str], hyp: Sequence[str]) -> int:
    """Levenshtein distance over words (substitution = deletion = insertion = 1)."""
    if not ref:
        return len(hyp)
    prev = list(range(len(hyp) + 1))
    for i, r in enumerate(ref, 1):
        cur = [i] + [0] * len(hyp)
        for j, h in enumerate(hyp, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (r != h))
        prev = cur
    return prev[-1]


def wer(predictions: Iterable[str], references: Iterable[str]) -> float:
    """Corpus WER in percent (jiwer: whitespace words, Σ errors / Σ reference words)."""
    errors = words = 0
    for p, r in zip(predictions, references):
        rw, pw = r.split(), p.split()
        errors += edit_distance(rw, pw)
        words += len(rw)
    return 100.0 * errors / max(words, 1)


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
        sd = st = 0
        for bw in (norm(w) for w in words):
            toks = bw.split()
            if not toks:
                continue
            rc = r.count(bw)
            if rc == 0:
                continue
            st += len(toks) * rc
            pc = p.count(bw)
            if pc != rc:
                sd += abs(rc - pc) * len(toks)
        if st > 0:
            total_d += sd
            total_t += st
    return {"bias_wer": 100.0 * total_d / total_t if total_t else 0.0, "bias_tokens": total_t}
