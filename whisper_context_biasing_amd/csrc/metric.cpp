// Host-side WER / bias-WER counting — the scoring half of BASELINE.json's
// metric, for batch scoring of whole evaluation splits.
//
// Restates the arithmetic of utils/compute_metric.py on already-normalised text (the Unicode
// normaliser stays in Python, metrics.py: BasicTextNormalizer, compute_metric.py:13-86):
//   * wcb_wer_counts — corpus WER as `evaluate.load("wer").compute` does for compute_metric.py:159
//     (jiwer): words = whitespace-separated tokens, Σ word-level Levenshtein distance
//     (substitution = insertion = deletion = 1) and Σ reference words. Utterances are scored in
//     parallel on host threads; each distance is an O(|ref|·|hyp|) two-row DP over word ids
//     (words interned per utterance, so the inner loop compares integers).
//   * wcb_bias_counts — compute_bias_wer's per-utterance tallies (compute_metric.py:200-230):
//     for each bias phrase, non-overlapping occurrence counts in the space-joined reference and
//     prediction (Python str.count, :216,222 — a byte-substring count is the same on UTF-8),
//     tokens += words(phrase)·ref_count, distance += |ref_count − pred_count|·words(phrase), phrases
//     absent from the reference skipped.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/wcb.h"

namespace {

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

std::vector<std::string_view> split_words(const char* s) {
  std::vector<std::string_view> w;
  const size_t n = std::strlen(s);
  size_t i = 0;
  while (i < n) {
    while (i < n && is_space(s[i])) ++i;
    const size_t j0 = i;
    while (i < n && !is_space(s[i])) ++i;
    if (i > j0) w.emplace_back(s + j0, i - j0);
  }
  return w;
}

int64_t word_distance(const char* ref, const char* hyp, int64_t* ref_words) {
  const auto r = split_words(ref), h = split_words(hyp);
  *ref_words = (int64_t)r.size();
  if (r.empty()) return (int64_t)h.size();
  if (h.empty()) return (int64_t)r.size();
  std::unordered_map<std::string_view, int> ids;
  std::vector<int> ri(r.size()), hi(h.size());
  for (size_t i = 0; i < r.size(); ++i) ri[i] = ids.emplace(r[i], (int)ids.size()).first->second;
  for (size_t j = 0; j < h.size(); ++j) hi[j] = ids.emplace(h[j], (int)ids.size()).first->second;
  std::vector<int64_t> prev(h.size() + 1), cur(h.size() + 1);
  for (size_t j = 0; j <= h.size(); ++j) prev[j] = (int64_t)j;
  for (size_t i = 1; i <= r.size(); ++i) {
    cur[0] = (int64_t)i;
    for (size_t j = 1; j <= h.size(); ++j)
      cur[j] = std::min({prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ri[i - 1] != hi[j - 1])});
    std::swap(prev, cur);
  }
  return prev[h.size()];
}

int64_t count_nonoverlapping(std::string_view hay, std::string_view needle) {
  int64_t c = 0;
  size_t p = 0;
  while ((p = hay.find(needle, p)) != std::string_view::npos) { ++c; p += needle.size(); }
  return c;
}

}  // namespace

extern "C" {

int wcb_wer_counts(const char* const* refs, const char* const* hyps, int n, int64_t* errors, int64_t* ref_words,
                   int n_threads) {
  if (n < 0 || (n > 0 && (!refs || !hyps || !errors || !ref_words))) return WCB_ERR_ARG;
  for (int i = 0; i < n; ++i)
    if (!refs[i] || !hyps[i]) return WCB_ERR_ARG;
  const int nt = std::max(1, std::min(n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency(),
                                      std::max(1, n / 16)));
  auto work = [&](int t) {
    for (int i = t; i < n; i += nt) errors[i] = word_distance(refs[i], hyps[i], &ref_words[i]);
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
  }
  return WCB_OK;
}

int wcb_bias_counts(const char* ref, const char* pred, const char* const* phrases, int n_phrases,
                    int64_t* distance, int64_t* tokens) {
  if (!ref || !pred || !distance || !tokens || n_phrases < 0 || (n_phrases > 0 && !phrases)) return WCB_ERR_ARG;
  const std::string_view r(ref), p(pred);
  int64_t sd = 0, st = 0;
  for (int k = 0; k < n_phrases; ++k) {
    if (!phrases[k]) return WCB_ERR_ARG;
    const auto toks = split_words(phrases[k]);
    if (toks.empty()) continue;
    const std::string_view bw(phrases[k]);
    const int64_t rc = count_nonoverlapping(r, bw);
    if (rc == 0) continue;
    st += (int64_t)toks.size() * rc;
    const int64_t pc = count_nonoverlapping(p, bw);
    if (pc != rc) sd += (rc > pc ? rc - pc : pc - rc) * (int64_t)toks.size();
  }
  *distance = sd;
  *tokens = st;
  return WCB_OK;
}

}  // extern "C"
