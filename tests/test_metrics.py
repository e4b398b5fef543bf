"""CPU: host-side WER / bias-WER against the values the reference's own formulas give on its
recorded outputs (results/*.txt + JSONL bias_words)."""
import gzip
import json
import os

import pytest

from whisper_context_biasing_amd.metrics import BasicTextNormalizer, bias_wer, parse_refs_preds, wer, wer_counts

GOLD = os.path.join(os.path.dirname(__file__), "golden")
EXPECT = {"dev": (8.330, 45.052, 13238), "test": (12.402, 57.287, 12844)}


@pytest.mark.parametrize("split", ["dev", "test"])
def test_reference_metric_goldens(split):
    d = json.load(gzip.open(os.path.join(GOLD, f"metric_{split}.json.gz"), "rt", encoding="utf-8"))
    refs, preds = parse_refs_preds(d["raw_lines"])
    assert len(refs) == len(d["bias_words"])
    w = wer(preds, refs)
    b = bias_wer(refs, preds, d["bias_words"])
    exp_w, exp_b, exp_tok = EXPECT[split]
    assert abs(w - exp_w) < 5e-3, w
    assert abs(b["bias_wer"] - exp_b) < 5e-3, b
    assert b["bias_tokens"] == exp_tok


def test_normalizer_and_distance():
    n = BasicTextNormalizer()
    assert n("Hello, World! [noise] (aside)  Done.") == "hello world done "
    assert wer_counts(["a x c d"], ["a b c"]) == ([2], [3])
    assert wer(["a b"], ["a b c"]) == pytest.approx(100 / 3)


def _py_edit_distance(ref, hyp):
    """Checker: the textbook word Levenshtein DP (jiwer's arithmetic), pure Python."""
    prev = list(range(len(hyp) + 1))
    for i, r in enumerate(ref, 1):
        cur = [i] + [0] * len(hyp)
        for j, h in enumerate(hyp, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (r != h))
        prev = cur
    return prev[-1]


def _py_bias_counts(r, p, phrases):
    """Checker: compute_bias_wer's per-utterance tallies (utils/compute_metric.py:200-230)."""
    sd = st = 0
    for bw in phrases:
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
    return sd, st


def test_cpp_scorer_matches_python_restatement():
    import ctypes as C
    import random
    from whisper_context_biasing_amd import _lib
    from whisper_context_biasing_amd.metrics import _cstrs
    rng = random.Random(3)
    vocab = ["a", "b", "c", "dé", "ü", "xyz", "nausea", "aa"]
    refs, hyps = [], []
    for _ in range(300):
        refs.append(" ".join(rng.choice(vocab) for _ in range(rng.randint(0, 12))))
        hyps.append(" ".join(rng.choice(vocab) for _ in range(rng.randint(0, 12))))
    for nt in (1, 4):
        err, words = wer_counts(hyps, refs, n_threads=nt)
        assert err == [_py_edit_distance(r.split(), h.split()) for r, h in zip(refs, hyps)]
        assert words == [len(r.split()) for r in refs]
    lib = _lib.load()
    for r, h in zip(refs[:100], hyps[:100]):
        phrases = [" ".join(rng.choice(vocab) for _ in range(rng.randint(0, 2))) for _ in range(6)] + ["a a", " b "]
        d, t = C.c_int64(), C.c_int64()
        assert lib.wcb_bias_counts(r.encode(), h.encode(), _cstrs(phrases), len(phrases), C.byref(d), C.byref(t)) == 0
        assert (d.value, t.value) == _py_bias_counts(r, h, phrases)
    assert wer_counts([], []) == ([], [])
    with pytest.raises(ValueError):
        wer_counts(["a"], [])
