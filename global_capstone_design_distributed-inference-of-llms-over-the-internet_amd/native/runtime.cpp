// Native host runtime for the stage executor (C++17, pybind11).
//
//  * PageAllocator  - KV page free list with double-free detection (the role of the
//                     vendored Petals MemoryCache, reference petals/server/memory_cache.py:26-225,
//                     without its cross-process pipe protocol: one process owns one GPU).
//  * build_meta     - per-step batch metadata for the paged kernels: positions, KV slots,
//                     per-query (sequence row, context length) and last-token rows, written
//                     straight into caller-owned (pinned) buffers.  This is the per-token host
//                     work of the hot decode loop (reference src/rpc_handler.py:109-147 builds
//                     position ids per request in Python).
//  * pack_frame / unpack_header - the zero-copy wire framing of the TCP data plane
//                     (magic, header length, payload lengths; little-endian).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

class PageAllocator {
 public:
  explicit PageAllocator(int64_t n) : n_(n), used_(n, 0) {
    if (n < 0) throw std::invalid_argument("negative page count");
    free_.reserve(n);
    for (int64_t i = n - 1; i >= 0; --i) free_.push_back((int32_t)i);
  }
  int64_t free_count() const { return (int64_t)free_.size(); }
  int64_t capacity() const { return n_; }
  py::object alloc(int64_t k) {
    if (k < 0) throw std::invalid_argument("negative request");
    if ((size_t)k > free_.size()) return py::none();
    std::vector<int32_t> out((size_t)k);
    for (int64_t i = 0; i < k; ++i) {
      out[i] = free_.back();
      free_.pop_back();
      used_[out[i]] = 1;
    }
    return py::cast(out);
  }
  void free(const std::vector<int32_t>& pages) {
    for (int32_t p : pages) {
      if (p < 0 || p >= n_) throw std::out_of_range("page id out of range");
      if (!used_[p]) throw std::runtime_error("double free of KV page " + std::to_string(p));
      used_[p] = 0;
      free_.push_back(p);
    }
  }

 private:
  int64_t n_;
  std::vector<uint8_t> used_;
  std::vector<int32_t> free_;
};

template <typename T, int F>
static T* mut(py::array_t<T, F>& a, int64_t need, const char* name) {
  if (a.size() < need) throw std::invalid_argument(std::string(name) + ": buffer too small");
  return a.mutable_data();
}

// Returns the number of tokens written.
int64_t build_meta(py::array_t<int32_t, py::array::c_style> rows, py::array_t<int32_t, py::array::c_style> starts,
                   py::array_t<int32_t, py::array::c_style> ntoks,
                   py::array_t<int32_t, py::array::c_style> block_table, int64_t page_size,
                   py::array_t<int64_t, py::array::c_style> positions, py::array_t<int64_t, py::array::c_style> slots,
                   py::array_t<int32_t, py::array::c_style> q_seq, py::array_t<int32_t, py::array::c_style> q_ctx,
                   py::array_t<int32_t, py::array::c_style> last_rows) {
  const int64_t S = rows.size();
  if (starts.size() != S || ntoks.size() != S) throw std::invalid_argument("rows/starts/ntoks length mismatch");
  if (block_table.ndim() != 2) throw std::invalid_argument("block_table must be 2-D");
  if (page_size <= 0 || (page_size & (page_size - 1))) throw std::invalid_argument("page_size power of two");
  const int64_t R = block_table.shape(0), P = block_table.shape(1);
  const int32_t* r = rows.data();
  const int32_t* s0 = starts.data();
  const int32_t* nt = ntoks.data();
  const int32_t* bt = block_table.data();
  int64_t T = 0;
  for (int64_t i = 0; i < S; ++i) {
    if (nt[i] < 0) throw std::invalid_argument("negative token count");
    T += nt[i];
  }
  int64_t* pos = mut(positions, T, "positions");
  int64_t* sl = mut(slots, T, "slots");
  int32_t* qs = mut(q_seq, T, "q_seq");
  int32_t* qc = mut(q_ctx, T, "q_ctx");
  int32_t* lr = mut(last_rows, S, "last_rows");
  int64_t t = 0;
  for (int64_t i = 0; i < S; ++i) {
    const int32_t row = r[i];
    if (row < 0 || row >= R) throw std::out_of_range("session row out of range");
    const int32_t* tab = bt + (int64_t)row * P;
    for (int32_t j = 0; j < nt[i]; ++j, ++t) {
      const int64_t p = (int64_t)s0[i] + j;
      const int64_t pg = p / page_size;
      if (pg >= P) throw std::out_of_range("position beyond the session's page table");
      const int32_t page = tab[pg];
      if (page < 0) throw std::runtime_error("unallocated KV page for position " + std::to_string(p));
      pos[t] = p;
      sl[t] = (int64_t)page * page_size + (p & (page_size - 1));
      qs[t] = row;
      qc[t] = (int32_t)(p + 1);
    }
    lr[i] = (int32_t)(t - 1);
  }
  return T;
}

// ---- wire framing: [magic u32 'MPF1'][header_len u32][n_payloads u32][payload_len u64 x n][header][payloads] ----
static const uint32_t kMagic = 0x3146504D;  // "MPF1"

py::bytes pack_prefix(py::bytes header, const std::vector<uint64_t>& payload_lens) {
  std::string h = header;
  std::string out;
  out.resize(12 + 8 * payload_lens.size());
  uint32_t hl = (uint32_t)h.size(), n = (uint32_t)payload_lens.size();
  std::memcpy(&out[0], &kMagic, 4);
  std::memcpy(&out[4], &hl, 4);
  std::memcpy(&out[8], &n, 4);
  for (size_t i = 0; i < payload_lens.size(); ++i) std::memcpy(&out[12 + 8 * i], &payload_lens[i], 8);
  out += h;
  return py::bytes(out);
}

py::tuple unpack_fixed(py::bytes prefix12) {
  std::string p = prefix12;
  if (p.size() != 12) throw std::invalid_argument("frame prefix must be 12 bytes");
  uint32_t magic, hl, n;
  std::memcpy(&magic, &p[0], 4);
  std::memcpy(&hl, &p[4], 4);
  std::memcpy(&n, &p[8], 4);
  if (magic != kMagic) throw std::runtime_error("bad frame magic");
  if (hl > (64u << 20) || n > 4096) throw std::runtime_error("frame header too large");
  return py::make_tuple(hl, n);
}

PYBIND11_MODULE(_mpamd_runtime, m) {
  m.doc() = "MI355X Mini-Petals native host runtime";
  py::class_<PageAllocator>(m, "PageAllocator")
      .def(py::init<int64_t>())
      .def("free_count", &PageAllocator::free_count)
      .def("capacity", &PageAllocator::capacity)
      .def("alloc", &PageAllocator::alloc)
      .def("free", &PageAllocator::free);
  m.def("build_meta", &build_meta, py::arg("rows"), py::arg("starts"), py::arg("ntoks"),
        py::arg("block_table").noconvert(), py::arg("page_size"), py::arg("positions").noconvert(),
        py::arg("slots").noconvert(), py::arg("q_seq").noconvert(), py::arg("q_ctx").noconvert(),
        py::arg("last_rows").noconvert());
  m.def("pack_prefix", &pack_prefix);
  m.def("unpack_fixed", &unpack_fixed);
}
