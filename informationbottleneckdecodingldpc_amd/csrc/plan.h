// Host-side planning of the decoders and the encoder: pure C++17, no HIP.
//
// Everything the C ABI derives on the host before a launch lives here — the edge index arrays
// (map_node_connections), the fast path's work orders and small-batch tasks, the float path's degree-2
// fold plan, the fused kernels' task tables and the encoder's substitution / factorisation plan — so the
// same code is built twice: into libibldpc.so (capi.hip includes this header) and, with AddressSanitizer
// and UndefinedBehaviorSanitizer, into the CPU-only checker tests/asan/plan_check.cpp
// (tests/test_cpu_host.py::test_host_planning_under_sanitizers).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

namespace ibl {

constexpr int kMaxD = 16;         // largest node degree with an unrolled fast-path body
constexpr int kLightD = 4;        // nodes up to this degree run with a 4-row item buffer
constexpr int kFoldRec = 8;       // ints per check of the float fold plan (FlArgs::fold)

// The host copy of a code graph (ibl_graph derives from it): CSR of H with its CSC-side arrays.
struct HostGraph {
  int32_t n_v = 0, n_c = 0;
  int64_t n_e = 0;
  std::vector<int32_t> h_cn_deg, h_vn_deg;
  std::vector<int32_t> h_cn_start, h_cols, h_vn_start, h_tgt_vn;
};

// Tanner-graph index construction (discrete_LDPC_decoder_irreg.py:121-170): canonical CSR in, the
// reference's start / degree / target arrays out. Returns false with *err set on malformed input.
inline bool map_node_connections(int32_t n_v, int32_t n_c, const int32_t* indptr, const int32_t* cols,
                                 int32_t* cn_start, int32_t* cn_deg, int32_t* tgt_cn, int32_t* vn_start,
                                 int32_t* vn_deg, int32_t* tgt_vn, std::string* err) {
  if (n_v <= 0 || n_c <= 0 || !indptr || !cols) return *err = "empty graph", false;
  if (indptr[0] != 0) return *err = "csr_indptr[0] must be 0", false;
  std::vector<int32_t> vdeg(n_v, 0);
  for (int32_t c = 0; c < n_c; ++c) {
    if (indptr[c + 1] < indptr[c]) return *err = "csr_indptr not monotone", false;
    for (int32_t e = indptr[c]; e < indptr[c + 1]; ++e) {
      if (cols[e] < 0 || cols[e] >= n_v) return *err = "column index out of range", false;
      if (e > indptr[c] && cols[e] <= cols[e - 1])
        return *err = "column indices must be strictly ascending within a row (canonical CSR)", false;
      vdeg[cols[e]]++;
    }
    cn_start[c] = indptr[c];
    cn_deg[c] = indptr[c + 1] - indptr[c];
  }
  int64_t acc = 0;
  for (int32_t v = 0; v < n_v; ++v) {
    vn_start[v] = (int32_t)acc;
    vn_deg[v] = vdeg[v];
    acc += vdeg[v];
  }
  // walking checks in ascending order fills each variable's edges in ascending row order
  std::vector<int64_t> fill(vn_start, vn_start + n_v);
  for (int32_t c = 0; c < n_c; ++c)
    for (int32_t e = indptr[c]; e < indptr[c + 1]; ++e) {
      const int64_t p = fill[cols[e]]++;
      tgt_cn[e] = (int32_t)p;
      tgt_vn[p] = e;
    }
  return true;
}

// Fast-path work order of one side: {node, first own-order edge, degree, 0} per position, heaviest first
// (stable); *heavy = positions of degree > kLightD.
inline std::vector<int32_t> work_order(const std::vector<int32_t>& start, const std::vector<int32_t>& deg,
                                       int32_t* heavy) {
  const int32_t n = (int32_t)deg.size();
  std::vector<int32_t> idx(n);
  for (int32_t i = 0; i < n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return deg[x] > deg[y]; });
  std::vector<int32_t> info(idx.size() * 4);
  *heavy = 0;
  for (size_t p = 0; p < idx.size(); ++p) {
    const int32_t v = idx[p];
    info[4 * p] = v;
    info[4 * p + 1] = start[v];
    info[4 * p + 2] = deg[v];
    info[4 * p + 3] = 0;
    if (deg[v] > kLightD) ++*heavy;
  }
  return info;
}

// {first position, count, degree, contiguous}: runs of at most 64 positions of one degree in a work order;
// contiguous = st0 + 1 when the run's nodes are consecutive and their own-order edges follow each other
// (node p0 + k at edge st0 + k·d), else 0 (the IB small-batch kernels then skip the per-lane record load)
inline std::vector<int32_t> order_tasks(const std::vector<int32_t>& info) {
  std::vector<int32_t> t;
  const int32_t n = (int32_t)(info.size() / 4);
  for (int32_t p = 0; p < n;) {
    const int32_t d = info[4 * p + 2];
    int32_t c = 0;
    while (p + c < n && c < 64 && info[4 * (p + c) + 2] == d) ++c;
    bool contig = true;
    for (int32_t k = 1; k < c && contig; ++k)
      contig = info[4 * (p + k)] == info[4 * p] + k && info[4 * (p + k) + 1] == info[4 * p + 1] + k * d;
    t.insert(t.end(), {p, c, d, contig ? info[4 * p + 1] + 1 : 0});
    p += c;
  }
  return t;
}

// Degree-2 variable fold (FlArgs::fold, fl_cn_item): a degree-2 variable v on checks c1, c2 is folded when
// both checks have one of their two fold slots free (variables taken in ascending order); each check's record
// names v's edge position in the check, the check-order row of v's other edge and v. Returns the folded
// variables' count; `rec` gets n_c records, `rest` the variables the variable pass still updates.
inline int32_t plan_fold(const HostGraph& g, std::vector<int32_t>* rec, std::vector<int32_t>* rest) {
  const int32_t nc = g.n_c, nv = g.n_v;
  rec->assign((size_t)nc * kFoldRec, 0);
  std::vector<int32_t> used(nc, 0);
  for (int32_t c = 0; c < nc; ++c) (*rec)[(size_t)kFoldRec * c] = (*rec)[(size_t)kFoldRec * c + 1] = -1;
  // check of each check-order edge
  std::vector<int32_t> chk_of(g.h_cols.size());
  for (int32_t c = 0; c < nc; ++c)
    for (int32_t k = 0; k < g.h_cn_deg[c]; ++k) chk_of[(size_t)g.h_cn_start[c] + k] = c;
  std::vector<char> folded(nv, 0);
  int32_t n = 0;
  for (int32_t v = 0; v < nv; ++v) {
    if (g.h_vn_deg[v] != 2) continue;
    const int32_t e1 = g.h_tgt_vn[(size_t)g.h_vn_start[v]], e2 = g.h_tgt_vn[(size_t)g.h_vn_start[v] + 1];
    const int32_t c1 = chk_of[(size_t)e1], c2 = chk_of[(size_t)e2];
    if (used[c1] >= 2 || used[c2] >= 2) continue;
    auto put = [&](int32_t c, int32_t e, int32_t other) {
      int32_t* r = &(*rec)[(size_t)kFoldRec * c];
      const int k = used[c]++;
      r[k] = e - g.h_cn_start[c];
      r[2 + k] = other;
      r[4 + k] = v;
    };
    put(c1, e1, e2);
    put(c2, e2, e1);
    folded[v] = 1;
    ++n;
  }
  rest->clear();
  for (int32_t v = 0; v < nv; ++v)
    if (!folded[v]) rest->push_back(v);
  return n;
}

// Task tables of the fused kernels (FlFusedArgs, IbFusedArgs).
struct FusedTasks {
  std::vector<int32_t> cn_task, vn_task, vn_node, vn_slot;
};

// Check nodes sorted by degree (heaviest first, stable) and cut into tasks of up to 64 nodes of one
// degree; edge k of lane i of a check task gets slot first + k*count + i. Variable nodes likewise;
// vn_slot maps each variable edge (task-major, k*count + i) to the slot of the same edge. bank_order
// reorders the variables of each degree for conflict-free dword slot reads, scanning `vwin` candidates per
// lane (below).
inline void build_fused_tasks(const HostGraph& g, FusedTasks* ft, bool bank_order, size_t vwin) {
  const int64_t E = g.n_e;
  vwin = std::max<size_t>(1, vwin);
  const std::vector<int32_t>& tgt_vn = g.h_tgt_vn;
  auto starts = [](const std::vector<int32_t>& deg) {
    std::vector<int64_t> st(deg.size() + 1, 0);
    for (size_t i = 0; i < deg.size(); ++i) st[i + 1] = st[i] + deg[i];
    return st;
  };
  auto sorted = [](const std::vector<int32_t>& deg) {
    std::vector<int32_t> idx(deg.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
    std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return deg[x] > deg[y]; });
    return idx;
  };
  const std::vector<int64_t> cst = starts(g.h_cn_deg), vst = starts(g.h_vn_deg);
  std::vector<int32_t> slot_of((size_t)E);
  {
    const std::vector<int32_t> ord = sorted(g.h_cn_deg);
    int32_t slot = 0;
    for (size_t i = 0; i < ord.size();) {
      const int32_t d = g.h_cn_deg[ord[i]];
      int32_t cnt = 0;
      while (i + cnt < ord.size() && cnt < 64 && g.h_cn_deg[ord[i + cnt]] == d) ++cnt;
      ft->cn_task.insert(ft->cn_task.end(), {slot, cnt, d, 0});
      for (int32_t l = 0; l < cnt; ++l)
        for (int32_t k = 0; k < d; ++k) slot_of[(size_t)cst[ord[i + l]] + k] = slot + k * cnt + l;
      slot += cnt * d;
      i += cnt;
    }
  }
  {
    std::vector<int32_t> ord = sorted(g.h_vn_deg);
    // Variable order within each degree: the variable pass reads its edge slots in check-task order,
    // so lanes of one 32-lane group (one LDS cycle of a ds_read_b32) collide when their k-th slots share
    // a bank (slot mod 32). Greedily fill each 32-lane group with variables whose k-th slots hit banks
    // not yet used by the group at that k (scan window vwin): the fused IB kernel's dword slots then read
    // (almost) conflict-free. Any order gives the same results.
    for (size_t i0 = 0; bank_order && i0 < ord.size();) {
      const int32_t d = g.h_vn_deg[ord[i0]];
      size_t i1 = i0;
      while (i1 < ord.size() && g.h_vn_deg[ord[i1]] == d) ++i1;
      std::vector<int32_t> pool(ord.begin() + (long)i0, ord.begin() + (long)i1), res;
      res.reserve(pool.size());
      auto bank = [&](int32_t v, int k) { return (uint32_t)slot_of[(size_t)tgt_vn[(size_t)vst[v] + k]] & 31u; };
      while (!pool.empty()) {
        uint32_t used[kMaxD + 1] = {0};
        for (int lane = 0; lane < 32 && !pool.empty(); ++lane) {
          size_t best = 0;
          int bestc = 1 << 30;
          const size_t win = std::min<size_t>(pool.size(), vwin);
          for (size_t c = 0; c < win && bestc > 0; ++c) {
            int col = 0;
            for (int k = 0; k < d && k <= kMaxD; ++k) col += (used[k] >> bank(pool[c], k)) & 1u;
            if (col < bestc) { bestc = col; best = c; }
          }
          const int32_t v = pool[best];
          for (int k = 0; k < d && k <= kMaxD; ++k) used[k] |= 1u << bank(v, k);
          res.push_back(v);
          pool.erase(pool.begin() + (long)best);
        }
      }
      std::copy(res.begin(), res.end(), ord.begin() + (long)i0);
      i0 = i1;
    }
    int32_t sidx = 0;
    for (size_t i = 0; i < ord.size();) {
      const int32_t d = g.h_vn_deg[ord[i]];
      int32_t cnt = 0;
      while (i + cnt < ord.size() && cnt < 64 && g.h_vn_deg[ord[i + cnt]] == d) ++cnt;
      ft->vn_task.insert(ft->vn_task.end(), {(int32_t)i, cnt, d, sidx});
      ft->vn_slot.resize((size_t)sidx + (size_t)cnt * d);
      for (int32_t l = 0; l < cnt; ++l) {
        const int32_t v = ord[i + l];
        ft->vn_node.push_back(v);
        for (int32_t k = 0; k < d; ++k) ft->vn_slot[(size_t)sidx + k * cnt + l] = slot_of[(size_t)tgt_vn[(size_t)vst[v] + k]];
      }
      sidx += cnt * d;
      i += cnt;
    }
  }
}

// The fused float kernel keeps the variable-edge slot indices in LDS as u16, each variable task's rows at the
// full stride of 64 lanes (record field 3 = the task's first padded index): the D index loads of a task share
// one address and take their row offsets as immediates, whatever the task's node count.
inline void pad_vn_slots(FusedTasks* ft) {
  std::vector<int32_t> pslot;
  for (size_t t = 0; t < ft->vn_task.size() / 4; ++t) {
    const int32_t cnt = ft->vn_task[4 * t + 1], d = ft->vn_task[4 * t + 2], sf = ft->vn_task[4 * t + 3];
    ft->vn_task[4 * t + 3] = (int32_t)pslot.size();
    for (int32_t k = 0; k < d; ++k)
      for (int32_t i = 0; i < 64; ++i) pslot.push_back(i < cnt ? ft->vn_slot[sf + (size_t)k * cnt + i] : 0);
  }
  ft->vn_slot.swap(pslot);
}

// ------------------------------------------------------------------ encoder plan
struct Csr {
  std::vector<int32_t> ip{0}, ix;
  void push_row(const std::vector<int32_t>& cols) {
    ix.insert(ix.end(), cols.begin(), cols.end());
    ip.push_back((int32_t)ix.size());
  }
};

// 1 lower / -1 upper triangular with full diagonal, 0 otherwise (LDPC_encoder.py:342-360);
// rows given as sorted column lists of the square parity part
inline int tri_shape(const std::vector<std::vector<int32_t>>& rows) {
  const int n = (int)rows.size();
  int64_t nnz = 0, low = 0;
  for (int i = 0; i < n; ++i) {
    bool diag = false;
    for (int c : rows[i]) {
      ++nnz;
      if (c <= i) ++low;
      if (c == i) diag = true;
    }
    if (!diag) return 0;
  }
  if (low == nnz) return 1;
  if (low == n) return -1;
  return 0;
}

// The plan getLDPCEncoderParamters (LDPC_encoder.py:197-269) derives from H = [A | B]: B triangular with a
// full diagonal (possibly after reversing its rows) -> forward / backward substitution over P = B's strict
// part; else GF(2) factorisation with gf2factorize's first-candidate pivot rule (:287-340) -> L, the pivot
// row order and P = strict upper part of U[piv]. chain = P is bidiagonal in substitution order (the prefix-
// XOR scan kernel).
struct EncPlan {
  std::string algo;
  int method = 0, dir = 1, chain = 0;   // method 1 = factorisation (L substitution first)
  Csr A, L, P;
  std::vector<int32_t> order;           // row order applied before P (empty: identity)
};

// Returns 0, -1 (malformed H), -2 (the parity part is singular in GF(2)) or -3 (too large to factorise); *err
// says which.
inline int encoder_plan(int32_t N, int32_t M, const int32_t* indptr, const int32_t* cols, EncPlan* pl,
                        std::string* err) {
  const int32_t K = N - M;
  std::vector<std::vector<int32_t>> brows(M);
  for (int32_t r = 0; r < M; ++r) {
    std::vector<int32_t> ac;
    for (int32_t e = indptr[r]; e < indptr[r + 1]; ++e) {
      const int32_t c = cols[e];
      if (c < 0 || c >= N) return *err = "column index out of range", -1;
      if (c < K) ac.push_back(c); else brows[r].push_back(c - K);
    }
    pl->A.push_row(ac);
  }
  auto strict = [&](const std::vector<std::vector<int32_t>>& rows, int dir) {
    Csr T;
    for (int i = 0; i < (int)rows.size(); ++i) {
      std::vector<int32_t> c;
      for (int j : rows[i])
        if (dir > 0 ? j < i : j > i) c.push_back(j);
      T.push_row(c);
    }
    return T;
  };
  int shape = tri_shape(brows);
  if (shape != 0) {                                    // (LDPC_encoder.py:208-213)
    pl->algo = shape == 1 ? "Forward Substitution" : "Backward Substitution";
    pl->dir = shape;
    pl->P = strict(brows, shape);
  } else {
    std::vector<std::vector<int32_t>> rev(brows.rbegin(), brows.rend());
    const int rshape = tri_shape(rev);
    if (rshape != 0) {                                 // rows reversed (:214-226)
      pl->algo = rshape == 1 ? "Forward Substitution" : "Backward Substitution";
      pl->dir = rshape;
      for (int i = 0; i < M; ++i) pl->order.push_back(M - 1 - i);
      pl->P = strict(rev, rshape);
    } else {                                           // GF(2) factorisation (:227-246, gf2factorize :287-340)
      if (M > 16384) return *err = "GF(2) factorisation limited to 16384 parity bits", -3;
      pl->algo = "Matrix Inverse";
      pl->method = 1;
      const int words = (M + 63) / 64;
      std::vector<uint64_t> Y2((size_t)M * words, 0), Y1((size_t)M * words, 0);
      for (int i = 0; i < M; ++i) {
        for (int c : brows[i]) Y2[(size_t)i * words + (c >> 6)] |= 1ull << (c & 63);
        Y1[(size_t)i * words + (i >> 6)] |= 1ull << (i & 63);
      }
      std::vector<char> used(M, 0);
      std::vector<int32_t> piv(M, 0);
      for (int col = 0; col < M; ++col) {
        const uint64_t bit = 1ull << (col & 63);
        int pv = -1;
        for (int i = 0; i < M; ++i)
          if (!used[i] && (Y2[(size_t)i * words + (col >> 6)] & bit)) {
            if (pv < 0) { pv = i; continue; }
            for (int w = 0; w < words; ++w) Y2[(size_t)i * words + w] ^= Y2[(size_t)pv * words + w];
            Y1[(size_t)i * words + (pv >> 6)] |= 1ull << (pv & 63);
          }
        if (pv < 0) return *err = "the last N-K columns of H are singular in GF(2)", -2;
        used[pv] = 1;
        piv[col] = pv;
      }
      auto row_cols = [&](const std::vector<uint64_t>& Y, int i) {
        std::vector<int32_t> c;
        for (int w = 0; w < words; ++w)
          for (uint64_t v = Y[(size_t)i * words + w]; v; v &= v - 1) c.push_back(w * 64 + __builtin_ctzll(v));
        return c;
      };
      std::vector<std::vector<int32_t>> l(M), u(M);
      for (int i = 0; i < M; ++i) {
        l[i] = row_cols(Y1, i);
        u[i] = row_cols(Y2, piv[i]);
      }
      pl->L = strict(l, 1);
      pl->P = strict(u, -1);
      pl->dir = -1;
      pl->order = piv;
    }
  }
  // bidiagonal P in substitution order -> prefix-XOR scan
  bool chain = true;
  for (int i = 0; i < M && chain; ++i) {
    const int n = pl->P.ip[i + 1] - pl->P.ip[i];
    const int want = pl->dir > 0 ? i - 1 : i + 1;
    if (want < 0 || want >= M) chain = n == 0;
    else chain = n == 1 && pl->P.ix[pl->P.ip[i]] == want;
  }
  pl->chain = chain ? 1 : 0;
  return 0;
}

}  // namespace ibl
