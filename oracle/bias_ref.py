"""Reference semantics of the bias-list log-prob boost — TEST ORACLE.

The reference has no inference-time boost; its biasing inputs are the per-item
`bias_words` (`data_utils/data_loader.py:163-167`) tokenised without special tokens. This module
DEFINES the operator the HIP path implements, as a pure-Python Aho-Corasick automaton:

* states = nodes of the trie of all phrase token sequences; root = 0;
* delta(s, v) = goto(s, v) following failure links (classic AC, full transition function);
* boosted(s, v)  <=>  delta(s, v) != root  (v extends a partial match or starts a phrase);
* greedy step: score[v] = logit[v] + lam * boosted(s, v); token = argmax (lowest index on ties);
  s <- delta(s, token).  lam == 0 gives plain greedy bit-for-bit.

Parity for lam > 0: unpinned (no reference implementation exists).
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Sequence


class AhoCorasick:
    def __init__(self, phrases: Sequence[Sequence[int]]):
        self.children: List[Dict[int, int]] = [{}]
        self.fail: List[int] = [0]
        self.depth: List[int] = [0]
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
                    self.children[s][int(v)] = nxt
                s = nxt
        # BFS failure links
        q = deque()
        for v, c in self.children[0].items():
            self.fail[c] = 0
            q.append(c)
        while q:
            s = q.popleft()
            for v, c in self.children[s].items():
                f = self.fail[s]
                while f and v not in self.children[f]:
                    f = self.fail[f]
                self.fail[c] = self.children[f].get(v, 0) if self.children[f].get(v, 0) != c else 0
                q.append(c)

    @property
    def n_states(self) -> int:
        return len(self.children)

    def delta(self, s: int, v: int) -> int:
        while True:
            c = self.children[s].get(v)
            if c is not None:
                return c
            if s == 0:
                return 0
            s = self.fail[s]

    def boosted_tokens(self, s: int) -> set:
        out = set()
        while True:
            out.update(self.children[s].keys())
            if s == 0:
                return out
            s = self.fail[s]


def boosted_argmax(logits_row, ac: AhoCorasick, state: int, lam: float, eos_mask: int = -1) -> int:
    """Argmax of logit + lam*boosted over one fp32 row, lowest index on ties."""
    import numpy as np
    row = np.asarray(logits_row, dtype=np.float32).copy()
    if lam != 0.0:
        for v in ac.boosted_tokens(state):
            row[v] = np.float32(row[v] + np.float32(lam))
    if eos_mask >= 0:
        row[eos_mask] = -np.inf
    return int(np.argmax(row))
