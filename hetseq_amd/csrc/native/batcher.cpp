// Native greedy batch sampler.
//
// Capability parity with the reference's Cython batcher
// (reference: data/data_utils_fast.pyx:10-61, data/data_utils.py:31-61):
// indices are packed in order into batches bounded by `max_sentences` and by
// `max_tokens` measured as (len(batch)+1) * max sample length, and an overfull
// batch is cut to a multiple of `bsz_mult` with the remainder carried over.
//
// Differences by design (MI355X-first host runtime):
//  * the per-index length comes from an int64 array (or a constant), never a
//    Python callback, so startup over millions of indices is a tight C++ loop;
//  * a constant-length fast path never materialises per-sample lengths;
//  * the output is a list of int64 numpy arrays (one per batch).
// The cut rule is reproduced exactly so the batch lists match the reference
// element for element (tests/test_data.py::test_batcher_* check golden lists).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct Cut {
  int64_t begin;
  int64_t end;
};

// Core loop: `len_of(i)` returns the token count of the i-th entry of `idx`.
template <typename LenFn>
std::vector<Cut> pack(const int64_t* idx, int64_t n, LenFn len_of, int64_t max_tokens,
                      int64_t max_sentences, int64_t bsz_mult) {
  std::vector<Cut> cuts;
  // Current batch is idx[b0, b1); the pending length list starts at l0 and
  // always covers [l0, i] (it already contains the candidate element, exactly
  // like the reference appends before testing for fullness).
  int64_t b0 = 0, b1 = 0, l0 = 0;
  int64_t sample_len = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t nt = len_of(i);
    sample_len = std::max(sample_len, nt);
    if (sample_len > max_tokens) {
      throw std::runtime_error("sentence at index " + std::to_string(idx[i]) + " of size " +
                               std::to_string(sample_len) + " exceeds max_tokens limit of " +
                               std::to_string(max_tokens) + "!");
    }
    const int64_t blen = b1 - b0;
    const int64_t num_tokens = (blen + 1) * sample_len;
    bool full = false;
    if (blen > 0) full = (blen == max_sentences) || (num_tokens > max_tokens);
    if (full) {
      const int64_t mod_len = std::max(bsz_mult * (blen / bsz_mult), blen % bsz_mult);
      cuts.push_back({b0, b0 + mod_len});
      b0 += mod_len;
      l0 += mod_len;
      sample_len = 0;
      for (int64_t j = l0; j <= i; ++j) sample_len = std::max(sample_len, len_of(j));
    }
    b1 = i + 1;
  }
  if (b1 > b0) cuts.push_back({b0, b1});
  return cuts;
}

py::list to_batches(const int64_t* idx, const std::vector<Cut>& cuts) {
  py::list out;
  for (const Cut& c : cuts) {
    py::array_t<int64_t> a(c.end - c.begin);
    std::copy(idx + c.begin, idx + c.end, a.mutable_data());
    out.append(std::move(a));
  }
  return out;
}

py::list batch_by_size(py::array_t<int64_t, py::array::c_style | py::array::forcecast> indices,
                       py::object num_tokens, int64_t max_tokens, int64_t max_sentences,
                       int64_t bsz_mult) {
  if (bsz_mult < 1) throw std::invalid_argument("required_batch_size_multiple must be >= 1");
  if (max_sentences < 1) throw std::invalid_argument("max_sentences must be >= 1");
  const int64_t n = indices.size();
  const int64_t* idx = indices.data();
  std::vector<Cut> cuts;
  if (py::isinstance<py::int_>(num_tokens)) {
    const int64_t c = num_tokens.cast<int64_t>();
    py::gil_scoped_release nogil;
    cuts = pack(idx, n, [c](int64_t) { return c; }, max_tokens, max_sentences, bsz_mult);
  } else {
    auto lens = num_tokens.cast<py::array_t<int64_t, py::array::c_style | py::array::forcecast>>();
    if (lens.size() != n) throw std::invalid_argument("num_tokens array must match indices length");
    const int64_t* l = lens.data();
    py::gil_scoped_release nogil;
    cuts = pack(idx, n, [l](int64_t i) { return l[i]; }, max_tokens, max_sentences, bsz_mult);
  }
  return to_batches(idx, cuts);
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "hetseq_amd native host runtime: batcher";
  m.def("batch_by_size", &batch_by_size, py::arg("indices"), py::arg("num_tokens"),
        py::arg("max_tokens"), py::arg("max_sentences"), py::arg("bsz_mult"),
        "Greedy size-bounded batching (reference-identical cut rule).");
}
