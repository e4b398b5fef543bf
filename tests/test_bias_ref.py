"""CPU: the A8 boost operator as oracle/bias_ref.py defines it — hand-worked transitions (extension,
retraction, banking of completed phrases, suffix re-matches, word-start gate), the potential identity
of the bonus over whole token streams, the vectorised row form against the per-token definition,
and that the boost raises the recall of bias phrases in a real greedy decode (numpy oracle, micro
model): phrases are the λ=0 decode's runner-up continuations, so λ=0 never emits them."""
import numpy as np
import pytest

from oracle import whisper_np as W
from oracle.bias_ref import AhoCorasick, boosted_argmax
from whisper_context_biasing_amd.config import get_dims
from whisper_context_biasing_amd.synth import synth_batch
from whisper_context_biasing_amd.weights import make_weights


def walk(ac, toks, s=0):
    units = []
    for v in toks:
        units.append(ac.units(s, v))
        s = ac.delta(s, v)
    return units, s


def test_hand_worked_transitions():
    ac = AhoCorasick([[1, 2, 3], [2, 5]])
    n1 = ac.delta(0, 1)
    n2 = ac.delta(n1, 2)
    n3 = ac.delta(n2, 3)
    assert [ac.depth[s] for s in (n1, n2, n3)] == [1, 2, 3] and ac.keep[n3] == 3 and ac.keep[n2] == 0
    assert ac.units(0, 1) == 1 and ac.units(0, 7) == 0       # start a phrase / nothing
    assert ac.units(n2, 3) == 1                              # extend
    assert ac.units(n2, 7) == -2                             # abandon "1 2": both bonuses retracted
    n5 = ac.delta(n2, 5)                                     # "1 2 5": suffix "2 5" completes
    assert ac.depth[n5] == 2 and ac.units(n2, 5) == 0        # drop "1" (-1), add "5" (+1)
    assert ac.units(n3, 7) == 0                              # completed "1 2 3": banked
    assert ac.units(n3, 1) == 1 and ac.delta(n3, 1) == n1    # banked, then a new start


def test_stream_totals():
    ac = AhoCorasick([[1, 2, 3], [2, 5], [4]])
    assert sum(walk(ac, [1, 2, 7])[0]) == 0                  # abandoned: as if never started
    assert sum(walk(ac, [1, 2, 3, 7, 7])[0]) == 3            # completed: lam per phrase token
    assert sum(walk(ac, [1, 2, 5, 7])[0]) == 2               # "1 2" abandoned, "2 5" completed
    assert sum(walk(ac, [4, 4, 1, 9])[0]) == 2               # two one-token phrases, one abandoned start


def test_longer_phrase_extends_a_completed_one():
    ac = AhoCorasick([[1], [1, 2, 3]])
    u, s = walk(ac, [1, 2, 9])
    assert u == [1, 1, -1] and s == 0                        # "1" kept, "2" of the unfinished "1 2 3" retracted
    u, s = walk(ac, [1, 2, 3, 9])
    assert sum(u) == 3


def test_potential_identity_without_completions():
    """With no phrase end reached, the summed units equal the depth of the final state."""
    rng = np.random.default_rng(0)
    phrases = [list(rng.integers(0, 6, size=rng.integers(2, 5))) for _ in range(12)]
    ac = AhoCorasick(phrases)
    checked = 0
    for _ in range(400):
        toks = list(rng.integers(0, 8, size=rng.integers(1, 12)))
        s, tot, completed = 0, 0, False
        for v in toks:
            tot += ac.units(s, v)
            s = ac.delta(s, v)
            completed |= ac.end[s] or ac.keep[s] > 0
        if not completed:
            assert tot == ac.depth[s], (toks, tot, ac.depth[s])
            checked += 1
    assert checked > 50


def test_word_start_gate():
    ws = np.ones(10, bool)
    ws[1] = False
    ac = AhoCorasick([[1, 2], [4, 1]], word_start=ws)
    assert ac.delta(0, 1) == 0 and ac.units(0, 1) == 0       # "1" cannot start a match
    n4 = ac.delta(0, 4)
    assert ac.depth[ac.delta(n4, 1)] == 2 and ac.units(n4, 1) == 1   # inside a match it may continue
    ac2 = AhoCorasick([[1, 2], [4, 1]])
    assert ac2.units(0, 1) == 1


@pytest.mark.parametrize("gate", [False, True])
def test_unit_vector_matches_definition(gate):
    rng = np.random.default_rng(1)
    V = 24
    phrases = [list(rng.integers(0, V, size=rng.integers(1, 5))) for _ in range(15)]
    ws = rng.random(V) < 0.5 if gate else None
    ac = AhoCorasick(phrases, ws)
    for s in range(ac.n_states):
        u = ac.unit_vector(s, V)
        assert [int(x) for x in u] == [ac.units(s, v) for v in range(V)]
    row = rng.standard_normal(V).astype(np.float32)
    for s in range(ac.n_states):
        ref = row + np.float32(2.0) * np.array([ac.units(s, v) for v in range(V)], np.float32)
        assert int(np.argmax(ref)) == boosted_argmax(row, ac, s, 2.0)


def runner_up_phrases(om, mel, n_tokens, lam, two_token=True):
    """Per row: at the step whose λ=0 top-1/top-2 logit gap is smallest (and below lam), the runner-up
    token r — and, with `two_token`, the greedy token after r (decode forced through r) — as a phrase."""
    ids, logits = om.generate(mel, max_length=n_tokens, min_new_tokens=n_tokens, return_logits=True, trim=False)
    phrases = []
    for b in range(ids.shape[0]):
        top2 = np.sort(logits[b], axis=-1)[:, -2:]
        gap = top2[:, 1] - top2[:, 0]
        t = int(np.argmin(gap[1:])) + 1                      # keep the first step (same start for every row)
        if gap[t] >= lam:
            continue
        r = int(np.argsort(logits[b, t])[-2])
        p = [r]
        if two_token:
            pre = [om.start] + [int(x) for x in ids[b, :t]] + [r]
            nxt = om.generate(mel[b:b + 1], max_length=1, min_new_tokens=1, prefix=pre, trim=False)
            p.append(int(nxt[0, 0]))
        phrases.append(p)
    return ids, phrases


def count_hits(ids, phrases):
    hits = 0
    for p in phrases:
        L = len(p)
        hits += sum(any(list(row[i:i + L]) == p for i in range(len(row) - L + 1)) for row in ids)
    return hits


def test_boost_raises_phrase_recall():
    dims = get_dims("micro")
    om = W.OracleModel.from_dims(dims, make_weights(dims, seed=0, recipe="diverse"))
    mel = W.log_mel(synth_batch(4), dims.n_mel)
    plain, phrases = runner_up_phrases(om, mel, 12, lam=2.0)
    assert len(phrases) >= 2
    boosted = om.generate(mel, max_length=12, min_new_tokens=12, bias=phrases, bias_boost=2.0, trim=False)
    h0, h1 = count_hits(plain, phrases), count_hits(boosted, phrases)
    assert h1 > h0 and h1 >= len(phrases) // 2, (h0, h1, phrases)
