"""CPU: host-side WER / bias-WER against the values the reference's own formulas give on its
recorded outputs (results/*.txt + JSONL bias_words)."""
import gzip
import json
import os

import pytest

from whisper_context_biasing_amd.metrics import BasicTextNormalizer, bias_wer, edit_distance, parse_refs_preds, wer

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
    assert edit_distance("a b c".split(), "a x c d".split()) == 2
    assert wer(["a b"], ["a b c"]) == pytest.approx(100 / 3)
