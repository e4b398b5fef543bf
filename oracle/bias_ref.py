"""Reference semantics of the bias-list log-prob boost — TEST ORACLE.

The reference has no inference-time boost; its biasing inputs are the per-item
`bias_words` (`data_utils/data_loader.py:163-167`) tokenised without special tokens. This module
DEFINES the operator the HIP path implements (k_select.hip, the LM-head epilogue, k_beam.hip), as
a pure-Python Aho-Corasick automaton with word-start gating and retraction of unfinished matches:

* states = nodes of the trie of all phrase token sequences, root = 0; depth(s) = trie depth;
  keep(s) = depth of the deepest phrase END on the trie path root..s (0 if none): the part of the
  current match that already completed a phrase.
* delta(s, v) = classic AC goto following failure links, except that a transition which would land
  on a depth-1 node (a match STARTING at v) requires word_start[v]; otherwise it lands on the root.
  `word_start` (a [V] bool mask, e.g. the tokens that begin with a space in a BPE vocabulary) is
  optional: None = every token may start a match.
* bonus units of token v in state s, with s' = delta(s, v), d = depth(s), k = keep(s), d' = depth(s'):
      n(s, v) = d' - d + min(k, d + 1 - d')
  i.e. +1 for every token that extends a match, minus the tokens of the current match that the
  transition drops and that did not complete a phrase (retraction); dropped tokens of a completed
  phrase stay credited. A hypothesis that starts a phrase and abandons it therefore ends with the
  same total bonus it would have had without starting it; a completed phrase keeps λ per token.
  Special cases: extending the match n = +1; falling back to the root n = k - d; starting a new
  phrase (gated root child) n = k - d + 1.
* score[v] = logit[v] + f32(lam) * f32(n(s, v))  (greedy: logits; beam: log-softmax; one f32
  product, one f32 add — the HIP kernels do exactly the same two roundings, no fused multiply-add),
  token = argmax (lowest index on ties), s <- delta(s, token). lam == 0 gives plain greedy / beam
  bit-for-bit (the kernels skip the add).

Parity for lam > 0: unpinned (no reference implementation exists); this restatement is the spec,
and tests/test_bias_ref.py checks it on hand-worked cases.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Optional, Sequence

import numpy as np


class AhoCorasick:
    def __init__(self, phrases: Sequence[Sequence[int]], word_start: Optional[Sequence[bool]] = None):
        self.children: List[Dict[int, int]] = [{}]
        self.fail: List[int] = [0]
        self.depth: List[int] = [0]
        self.end: List[bool] = [False]
        self.word_start = None if word_start is None else np.asarray(word_start, dtype=bool)
        for p in phrases:
            if len(p) == 0:
                continue
            s = 0
            for v in p:
                nxt = self.children[s].get(int(v))
                if nxt is None:
                    nxt = len(self.children)
                    self.children.append({})
                    self.fail.append(0)
                    self.depth.append(self.depth[s] + 1)
                    self.end.append(False)
                    self.children[s][int(v)] = nxt
                s = nxt
            self.end[s] = True
        # keep(s): deepest phrase end on the trie path (parents precede children in BFS order)
        self.keep: List[int] = [0] * len(self.children)
        q = deque()
        for v, c in self.children[0].items():
            self.fail[c] = 0
            q.append(c)
        for c in q:
            self.keep[c] = self.depth[c] if self.end[c] else 0
        while q:   # BFS failure links + keep
            s = q.popleft()
            for v, c in self.children[s].items():
                f = self.fail[s]
                while f and v not in self.children[f]:
                    f = self.fail[f]
                self.fail[c] = self.children[f].get(v, 0) if self.children[f].get(v, 0) != c else 0
                self.keep[c] = self.depth[c] if self.end[c] else self.keep[s]
                q.append(c)
        self._units: Dict[int, np.ndarray] = {}

    @property
    def n_states(self) -> int:
        return len(self.children)

    def starts_word(self, v: int) -> bool:
        return self.word_start is None or bool(self.word_start[v])

    def delta(self, s: int, v: int) -> int:
        while True:
            c = self.children[s].get(v)
            if c is not None:
                return c if (s != 0 or self.starts_word(v)) else 0
            if s == 0:
                return 0
            s = self.fail[s]

    def units(self, s: int, v: int) -> int:
        """n(s, v): the bonus of token v in state s, in units of lam."""
        d, k = self.depth[s], self.keep[s]
        d2 = self.depth[self.delta(s, v)]
        return d2 - d + min(k, d + 1 - d2)

    def unit_vector(self, s: int, V: int) -> np.ndarray:
        """n(s, v) for every v < V (int32), cached per state: k - d everywhere, +1 on the gated root
        children, the exact value on the tokens whose transition lands deeper than depth 1."""
        u = self._units.get(s)
        if u is None or u.shape[0] != V:
            d, k = self.depth[s], self.keep[s]
            u = np.full(V, k - d, dtype=np.int32)
            for v in self.children[0]:
                if v < V and self.starts_word(v):
                    u[v] = k - d + 1
            f = s
            seen = set()
            while f:
                for v, c in self.children[f].items():
                    if v not in seen and v < V:
                        seen.add(v)
                        u[v] = self.units(s, v)
                f = self.fail[f]
            self._units[s] = u
        return u

    def boost_row(self, row: np.ndarray, s: int, lam: float) -> np.ndarray:
        """f32 row + f32(lam) * f32(n(s, .)) — two roundings, as the kernels compute it."""
        u = self.unit_vector(s, row.shape[-1]).astype(np.float32)
        return (np.asarray(row, dtype=np.float32) + np.float32(lam) * u).astype(np.float32)

    def boosted_tokens(self, s: int) -> set:
        """Tokens whose transition from s extends or starts a match (delta lands off the root)."""
        out = set()
        f = s
        while True:
            for v, c in self.children[f].items():
                if self.delta(s, v) != 0:
                    out.add(v)
            if f == 0:
                return out
            f = self.fail[f]


def boosted_argmax(logits_row, ac: AhoCorasick, state: int, lam: float, eos_mask: int = -1) -> int:
    """Argmax of logit + lam*n(state, .) over one fp32 row, lowest index on ties."""
    row = np.asarray(logits_row, dtype=np.float32)
    if lam != 0.0:
        row = ac.boost_row(row, state, lam)
    else:
        row = row.copy()
    if eos_mask >= 0:
        row[eos_mask] = -np.inf
    return int(np.argmax(row))
