// C ABI (include/ibldpc.h): handle management, table preparation and the decode schedules.
//
// Schedules restate the reference's host loops without their per-iteration host sync:
//   IB:    decode_OpenCL            (Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py:245-341)
//   float: decode_OpenCL_min_sum    (Continous_LDPC_Decoding/min_sum_decoder_irreg.py:221-287)
//          decode_OpenCL_belief_propagation (bp_decoder_irreg.py:221-286)
// Early stop: each check-node pass ORs "some check unsatisfied" into 64 flag words of its
// iteration; the launches of the next iteration read those words and exit at once when they
// are all zero, and a one-wave kernel turns the flags into the iteration index the output
// pass uses.  The host only enqueues.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <functional>
#include <map>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "ibldpc.h"

using namespace ibl;

// IBL_DIAG=1 (diagnostic builds, tools/variants.py): the timing-only hooks IBL_VN_PART, IBL_TRACE_WAVES and
// IBL_TRACE_FUSED, and IBL_ALLOW_SCRATCH (create accepts a fast-path build with a private segment). The product
// build has none of them: no decode call reads the environment, and create always refuses scratch.
#ifndef IBL_DIAG
#define IBL_DIAG 0
#endif

static thread_local std::string g_err;
static inline void dfree(void* p) {
  if (p) (void)hipFree(p);
}

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int ibl::set_error(int code, const char* msg) { return fail(code, msg ? msg : ""); }
// Diagnostic builds: IBL_DEBUG_SYNC=1 synchronises after every launch so an asynchronous fault is
// reported at the launch that caused it (breaks the no-host-sync property of decode).
static bool debug_sync() {
#if IBL_DIAG
  static const bool on = [] {
    const char* v = getenv("IBL_DEBUG_SYNC");
    return v && *v && *v != '0';
  }();
  return on;
#else
  return false;
#endif
}
#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e == hipSuccess && debug_sync()) _e = hipDeviceSynchronize();                      \
    if (_e != hipSuccess)                                                                   \
      return fail(IBL_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)

template <typename T>
static int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return fail(IBL_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return IBL_OK;
}
template <typename T>
static int dupload(T** p, const T* h, size_t count) {
  int rc = dalloc(p, count);
  if (rc) return rc;
  if (count) HIPCHK(hipMemcpy(*p, h, count * sizeof(T), hipMemcpyHostToDevice));
  return IBL_OK;
}

struct ibl_graph : HostGraph {   // host copies (plan.h: fold / fused task set-up) + the device arrays
  int device = 0, num_cus = 256;
  int32_t dcm = 0, dvm = 0;
  int32_t *cn_start = nullptr, *cn_deg = nullptr, *tgt_cn = nullptr;
  int32_t *vn_start = nullptr, *vn_deg = nullptr, *tgt_vn = nullptr, *csr_cols = nullptr;
  // fast-path work order: {node, start, degree, 0} per position, heaviest first (stable)
  int32_t *cn_info = nullptr, *vn_info = nullptr;
  int32_t cn_heavy = 0, vn_heavy = 0;
  // small-batch kernels: tasks of up to 64 consecutive same-degree positions of cn_info / vn_info
  int32_t *cn_task = nullptr, *vn_task = nullptr;
  int32_t n_cn_task = 0, n_vn_task = 0;
};


// HIP-event timing of the CN / VN launches (benchmark only).
struct KTimer {
  bool on = false;
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<int, int>> pending;  // (kind 0=CN 1=VN, first event index)
  size_t next = 0;
  int mark(hipStream_t s) {
    if (next == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return -1;
      pool.push_back(e);
    }
    (void)hipEventRecord(pool[next], s);
    return (int)next++;
  }
  template <typename F>
  hipError_t timed(int kind, hipStream_t s, F&& launch) {
    if (!on) return launch();
    const int a = mark(s);
    hipError_t e = launch();
    mark(s);
    if (a >= 0) pending.emplace_back(kind, a);
    return e;
  }
  int read(double* cn_ms, int32_t* cn_n, double* vn_ms, int32_t* vn_n) {
    double ms[2] = {0, 0};
    int32_t n[2] = {0, 0};
    for (auto& p : pending) {
      if (hipEventSynchronize(pool[p.second + 1]) != hipSuccess) return -1;
      float t = 0.f;
      if (hipEventElapsedTime(&t, pool[p.second], pool[p.second + 1]) != hipSuccess) return -1;
      ms[p.first] += t;
      n[p.first] += 1;
    }
    pending.clear();
    next = 0;
    if (cn_ms) *cn_ms = ms[0];
    if (cn_n) *cn_n = n[0];
    if (vn_ms) *vn_ms = ms[1];
    if (vn_n) *vn_n = n[1];
    return 0;
  }
  ~KTimer() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

struct KCfg {
  int grid = 0, block = 256;
  size_t lds = 0;
};

// Small-batch pass chains replayed from captured graphs. A decode of a few codewords is ~2 i_max dependent launches
// of a few microseconds each; launching them one by one costs the host about as much as the GPU spends running
// them, so a caller that does anything else per batch (the BER driver) leaves the GPU waiting. The chain between
// channel staging and the stop-iteration / decision kernels touches only the decoder's own buffers, so it is
// captured once per (batch, early stop) on a private stream and replayed on the caller's stream with one call.
struct ChainGraphs {
  hipStream_t cap = nullptr;
  std::map<std::pair<int, int>, hipGraphExec_t> execs;
  bool on = false;
  void clear() {
    for (auto& e : execs) (void)hipGraphExecDestroy(e.second);
    execs.clear();
  }
  ~ChainGraphs() {
    clear();
    if (cap) (void)hipStreamDestroy(cap);
  }
  // run chain(stream) for key on stream s: replay its graph, capturing it first if needed
  template <class F>
  hipError_t run(int B, int early, hipStream_t s, F&& chain) {
    const auto key = std::make_pair(B, early);
    auto it = execs.find(key);
    if (it == execs.end()) {
      if (!cap) {
        const hipError_t e = hipStreamCreateWithFlags(&cap, hipStreamNonBlocking);
        if (e != hipSuccess) return e;
      }
      if (execs.size() >= 64) clear();   // bounded: at most 64 batch sizes kept
      hipError_t e = hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal);
      if (e != hipSuccess) return e;
      const hipError_t ec = chain(cap);
      hipGraph_t graph = nullptr;
      e = hipStreamEndCapture(cap, &graph);
      if (ec != hipSuccess || e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return ec != hipSuccess ? ec : e;
      }
      hipGraphExec_t exec = nullptr;
      e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
      (void)hipGraphDestroy(graph);
      if (e != hipSuccess) return e;
      it = execs.emplace(key, exec).first;
    }
    return hipGraphLaunch(it->second, s);
  }
};

struct ibl_ib {
  const ibl_graph* g = nullptr;
  int32_t Tc = 0, T = 0, imax = 0, CM = 0, VM = 0, match = 0, max_batch = 0, ldb = 0;
  bool fast = false;
  uint8_t *cin = nullptr, *vin = nullptr, *ch8 = nullptr;
  int32_t *flags = nullptr, *dL = nullptr;
  // fast path
  uint32_t *cn_img = nullptr, *vn_img = nullptr, *dec_img = nullptr;
  int cn_nt = 0, vn_nt = 0, dec_nt = 0;   // fast path: LDS table quads (4 tables each) per pass
  int32_t cn_fslot[kMaxD + 1] = {0}, vn_fslot[kMaxD + 1] = {0};
  uint32_t *cn_cimg = nullptr, *vn_cimg = nullptr;   // column images per pass (ncs x 32 dwords)
  int cn_ncs = 0, vn_ncs = 0;
  int8_t cn_ccol[kMaxD + 1][4] = {{0}}, vn_ccol[kMaxD + 1][4] = {{0}};
  KCfg kcn, kvn, kdec;
  KTimer timer;
  // fused on-chip path (IbFusedArgs, short codes): task tables, LDS bytes per workgroup, grid
  int32_t path = IBL_PATH_AUTO;
  bool fused_ok = false, f_half_ok = false;   // f_half_ok: the 4-codeword-group kernel is usable too
  int32_t f_ncw_forced = 0;                   // IBL_FUSED_NCW read once at create (A/B, tests), 0 = auto
  // small-batch per-pass kernels (ib_*_small) for B <= small_b (0: off); LDS bytes per launch kind
  int32_t small_b = 0;
  bool s_ok = false;                          // the small-batch kernels exist for this decoder and run without scratch
  size_t s_lds_cn = 0, s_lds_vn = 0, s_lds_dec = 0;
  ChainGraphs s_graphs;                       // small-batch pass chains (IBL_SMALL_GRAPH=0 at create: launch them)
  int32_t *f_cn_task = nullptr, *f_vn_task = nullptr, *f_vn_node = nullptr, *f_vn_slot = nullptr;
  int32_t f_ncn = 0, f_nvn = 0, f_nreg = 0, f_dbuf = 0, f_cn_uni = 0, f_vn_uni = 0;
  size_t f_lds = 0;
  int f_grid = 0, f_block = 0;
  // generic path
  int32_t *cn_lut = nullptr, *vn_lut = nullptr, *mc = nullptr, *mv = nullptr;
  int64_t cn_len = 0, vn_len = 0, mc_len = 0, mv_len = 0;
};

struct ibl_float {
  const ibl_graph* g = nullptr;
  int32_t kind = 0, imax = 0, prec = kF32, max_batch = 0, ldb = 0;
  double llr_max = 150.0;
  void *cin = nullptr, *vbuf0 = nullptr, *vbuf1 = nullptr, *chf = nullptr;
  int32_t *flags = nullptr, *dL = nullptr;
  int grid_cn = 0, grid_vn = 0;
  // degree-2 variable fold of the per-pass path (fl_cn_item): per-check records, the variables the
  // variable pass still updates, the second check inbox (the check passes alternate between cin / cin2)
  void* cin2 = nullptr;
  int32_t *fold = nullptr, *vn_nodes = nullptr;
  int32_t n_vn_nodes = 0, n_folded = 0;
  std::vector<int32_t> fold_rec, fold_rest;   // the fold's host plan; uploaded with cin2 once a batch can use it
  int32_t* bad = nullptr;   // channel LLRs that violated the precondition since the last ibl_float_input_check
  int32_t small_b = 0;      // small-batch kernels (fl_*_small) for B <= small_b (0: off)
  bool s_ok = false;        // the small-batch kernels run without scratch (create's check)
  ChainGraphs s_graphs;     // small-batch pass chains (IBL_SMALL_GRAPH=0 at create: launch them one by one)
  KTimer timer;
  // fused on-chip path (FlFusedArgs): task tables, LDS bytes per workgroup, grid
  int32_t path = IBL_PATH_AUTO;
  bool fused_ok = false;
  int32_t *f_cn_task = nullptr, *f_vn_task = nullptr, *f_vn_node = nullptr, *f_vn_slot = nullptr;
  int32_t f_ncn = 0, f_nvn = 0, f_nvs = 0;
  size_t f_lds = 0;
  int f_grid = 0;
};

extern "C" {

int ibl_version(void) { return IBL_VERSION; }
const char* ibl_last_error(void) { return g_err.c_str(); }

int ibl_device_count(int32_t* n) {
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (n) *n = (e == hipSuccess) ? c : 0;
  return IBL_OK;
}

int ibl_map_node_connections(int32_t n_v, int32_t n_c, const int32_t* indptr, const int32_t* cols,
                             int32_t* cn_start, int32_t* cn_deg, int32_t* tgt_cn, int32_t* vn_start,
                             int32_t* vn_deg, int32_t* tgt_vn) {
  std::string err;
  if (!map_node_connections(n_v, n_c, indptr, cols, cn_start, cn_deg, tgt_cn, vn_start, vn_deg, tgt_vn, &err))
    return fail(IBL_EINVAL, err);
  return IBL_OK;
}

int ibl_graph_create(int32_t n_v, int32_t n_c, const int32_t* indptr, const int32_t* cols, int32_t device,
                     ibl_graph** out) {
  if (!out) return fail(IBL_EINVAL, "out is NULL");
  *out = nullptr;
  if (n_v <= 0 || n_c <= 0) return fail(IBL_EINVAL, "empty graph");
  const int64_t E = indptr[n_c];
  std::vector<int32_t> cs(n_c), cd(n_c), tc(E), vs(n_v), vd(n_v), tv(E);
  int rc = ibl_map_node_connections(n_v, n_c, indptr, cols, cs.data(), cd.data(), tc.data(), vs.data(), vd.data(),
                                    tv.data());
  if (rc) return rc;
  for (int32_t c = 0; c < n_c; ++c)
    if (cd[c] < 2 || cd[c] > 255) return fail(IBL_EUNSUPPORTED, "check-node degrees must lie in [2, 255]");
  for (int32_t v = 0; v < n_v; ++v)
    if (vd[v] < 1 || vd[v] > 255) return fail(IBL_EUNSUPPORTED, "variable-node degrees must lie in [1, 255]");
  HIPCHK(hipSetDevice(device));
  auto* g = new ibl_graph();
  g->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) g->num_cus = prop.multiProcessorCount;
  g->n_v = n_v;
  g->n_c = n_c;
  g->n_e = E;
  g->dcm = *std::max_element(cd.begin(), cd.end());
  g->dvm = *std::max_element(vd.begin(), vd.end());
  g->h_cn_deg = cd;
  g->h_vn_deg = vd;
  g->h_cn_start = cs;
  g->h_cols.assign(cols, cols + E);
  g->h_vn_start = vs;
  g->h_tgt_vn = tv;
  if ((rc = dupload(&g->cn_start, cs.data(), n_c)) || (rc = dupload(&g->cn_deg, cd.data(), n_c)) ||
      (rc = dupload(&g->tgt_cn, tc.data(), E)) || (rc = dupload(&g->vn_start, vs.data(), n_v)) ||
      (rc = dupload(&g->vn_deg, vd.data(), n_v)) || (rc = dupload(&g->tgt_vn, tv.data(), E)) ||
      (rc = dupload(&g->csr_cols, cols, E))) {
    ibl_graph_destroy(g);
    return rc;
  }
  {
    const std::vector<int32_t> ci = work_order(cs, cd, &g->cn_heavy), vi = work_order(vs, vd, &g->vn_heavy);
    const std::vector<int32_t> ct = order_tasks(ci), vt = order_tasks(vi);
    g->n_cn_task = (int32_t)(ct.size() / 4);
    g->n_vn_task = (int32_t)(vt.size() / 4);
    if ((rc = dupload(&g->cn_info, ci.data(), ci.size())) || (rc = dupload(&g->vn_info, vi.data(), vi.size())) ||
        (rc = dupload(&g->cn_task, ct.data(), ct.size())) || (rc = dupload(&g->vn_task, vt.data(), vt.size()))) {
      ibl_graph_destroy(g);
      return rc;
    }
  }
  *out = g;
  return IBL_OK;
}

int ibl_graph_info(const ibl_graph* g, int32_t* n_v, int32_t* n_c, int64_t* n_e, int32_t* dcm, int32_t* dvm) {
  if (!g) return fail(IBL_EINVAL, "graph is NULL");
  if (n_v) *n_v = g->n_v;
  if (n_c) *n_c = g->n_c;
  if (n_e) *n_e = g->n_e;
  if (dcm) *dcm = g->dcm;
  if (dvm) *dvm = g->dvm;
  return IBL_OK;
}

void ibl_graph_destroy(ibl_graph* g) {
  if (!g) return;
  (void)hipSetDevice(g->device);
  dfree(g->cn_start); dfree(g->cn_deg); dfree(g->tgt_cn);
  dfree(g->vn_start); dfree(g->vn_deg); dfree(g->tgt_vn); dfree(g->csr_cols);
  dfree(g->cn_info); dfree(g->vn_info); dfree(g->cn_task); dfree(g->vn_task);
  delete g;
}

}  // extern "C"

// ------------------------------------------------------------------ IB table images
namespace {

using Table = std::vector<uint8_t>;  // 256 entries, (t, m) at t*16 + m

Table make_table(int T, const std::function<int(int, int)>& f) {
  Table tb(256, 0);
  for (int t = 0; t < T; ++t)
    for (int m = 0; m < T; ++m) tb[t * kTP + m] = (uint8_t)f(t, m);
  return tb;
}

// One pass's tables as quads (common.h): nreg x 256 dwords, dword (t*16+m) of quad R holds entry (t, m)
// of table 4R+j in byte j (slot_off); the kernels replicate each dword over the 32 banks. Unused slots
// of the last quad are 0.
void append_pass(std::vector<uint32_t>& img, const std::vector<Table>& tbs, int nreg) {
  for (int R = 0; R < nreg; ++R)
    for (int r = 0; r < 256; ++r) {
      uint32_t w = 0;
      for (int j = 0; j < 4; ++j) {
        const size_t k = (size_t)4 * R + j;
        if (k < tbs.size()) w |= (uint32_t)tbs[k][r] << (8 * j);
      }
      img.push_back(w);
    }
}

std::vector<int> present(const std::vector<int32_t>& deg) {
  std::vector<int> d(deg.begin(), deg.end());
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  return d;
}

// LDS bytes of a fast CN / VN launch: table quads, column images, the 2 work counters
size_t fast_lds(int nt, int ncs) {
  return lds_of_quads(regions_of(nt)) + (size_t)ncs * kColImg + 64;
}

// One pass's column images (colf): per image slot, 16 columns m x {entries t = 0..7, t = 8..15} as nibbles
void append_cols(std::vector<uint32_t>& img, const std::vector<Table>& tbs, const std::vector<int>& slots) {
  for (int s : slots)
    for (int m = 0; m < kTP; ++m) {
      uint32_t lo = 0, hi = 0;
      for (int t = 0; t < 8; ++t) {
        lo |= (uint32_t)(tbs[s][t * kTP + m] & 15) << (4 * t);
        hi |= (uint32_t)(tbs[s][(t + 8) * kTP + m] & 15) << (4 * t);
      }
      img.push_back(lo);
      img.push_back(hi);
    }
}

int pick_cfg(int which, int maxd, int nt, int ncs, int num_cus, KCfg* k) {
  k->lds = fast_lds(nt, ncs);
  int best_waves = 0;
  // largest block first at equal occupancy: a CU's waves then share one work counter
  for (int block : {1024, 768, 640, 512, 384, 256}) {
    int bpc = 0;
    if (ib_fast_occupancy(which, maxd, block, k->lds, &bpc) != hipSuccess) continue;
    const int waves = bpc * block / 64;
    if (bpc > 0 && waves > best_waves) {
      best_waves = waves;
      k->block = block;
      k->grid = bpc * num_cus;
    }
  }
  return best_waves > 0 ? IBL_OK : fail(IBL_EHIP, "no occupancy for IB kernel (LDS too large?)");
}

int ib_fused_setup(ibl_ib* h);           // fused on-chip IB decoder (defined with the float one below)
bool ib_fused_in_use(const ibl_ib* h);

// Codewords per workgroup of the fused IB kernel for a batch of B: 4-codeword half groups when even the
// doubled number of workgroups fits the grid (each half group then has a workgroup slot of its own);
// whole 8-codeword groups otherwise — with 2*ngroups > grid some workgroups would run two half groups in
// a row, and a half group takes more than half a group's time (per-phase latency). The
// environment IBL_FUSED_NCW=8 / 4, read once when the decoder is created, forces either (A/B, tests); 4
// needs the half-group kernel (f_half_ok).
int ib_fused_ncw(const ibl_ib* h, int B) {
  const int ngroups = (B + 7) / 8;
  const int forced = h->f_ncw_forced;
  if (!h->f_half_ok || forced == 8) return 8;
  return (forced == 4 || 2 * ngroups <= h->f_grid) ? 4 : 8;
}
}  // namespace

extern "C" {

int ibl_ib_create(const ibl_graph* g, int32_t Tc, int32_t T, int32_t imax, const int32_t* cn_lut, int64_t cn_len,
                  const int32_t* vn_lut, int64_t vn_len, const int32_t* match_cn, int64_t mc_len,
                  const int32_t* match_vn, int64_t mv_len, int32_t match, int32_t max_batch, int32_t flags,
                  ibl_ib** out) {
  if (!out) return fail(IBL_EINVAL, "out is NULL");
  *out = nullptr;
  if (!g) return fail(IBL_EINVAL, "graph is NULL");
  if (Tc < 2 || T < 2 || Tc > 256 || T > 256) return fail(IBL_EUNSUPPORTED, "cardinalities must lie in [2, 256]");
  if (imax < 1) return fail(IBL_EINVAL, "imax must be >= 1");
  if (max_batch < 1) return fail(IBL_EINVAL, "max_batch must be >= 1");
  const int CM = g->dcm, VM = g->dvm;
  if (CM < 3) return fail(IBL_EUNSUPPORTED, "IB decoding needs a check-node degree >= 3");
  const int64_t need_cn = (int64_t)Tc * Tc + (int64_t)(CM - 3) * Tc * T + (int64_t)(imax - 1) * (CM - 2) * T * T;
  const int64_t need_vn = (int64_t)imax * ((int64_t)Tc * T + (int64_t)(VM - 1) * T * T);
  if (!cn_lut || cn_len < need_cn) return fail(IBL_EINVAL, "CN LUT vector shorter than the reference layout");
  if (!vn_lut || vn_len < need_vn) return fail(IBL_EINVAL, "VN LUT vector shorter than the reference layout");
  for (int64_t i = 0; i < cn_len; ++i)
    if (cn_lut[i] < 0 || cn_lut[i] >= T) return fail(IBL_EINVAL, "CN LUT entries must lie in [0, T_dec)");
  for (int64_t i = 0; i < vn_len; ++i)
    if (vn_lut[i] < 0 || vn_lut[i] >= T) return fail(IBL_EINVAL, "VN LUT entries must lie in [0, T_dec)");
  if (match) {
    if (!match_cn || mc_len < (int64_t)imax * CM * T || !match_vn || mv_len < (int64_t)imax * VM * T)
      return fail(IBL_EINVAL, "matching vectors shorter than (imax, d_max, T_dec)");
    for (int64_t i = 0; i < mc_len; ++i)
      if (match_cn[i] < 0 || match_cn[i] >= T) return fail(IBL_EINVAL, "matching entries must lie in [0, T_dec)");
    for (int64_t i = 0; i < mv_len; ++i)
      if (match_vn[i] < 0 || match_vn[i] >= T) return fail(IBL_EINVAL, "matching entries must lie in [0, T_dec)");
  }
  HIPCHK(hipSetDevice(g->device));
  auto* h = new ibl_ib();
  h->g = g;
  h->Tc = Tc; h->T = T; h->imax = imax; h->CM = CM; h->VM = VM; h->match = match ? 1 : 0;
  h->max_batch = max_batch;
  h->ldb = (max_batch + kRowPad - 1) / kRowPad * kRowPad;   // codewords; fast path rows = ldb/2 bytes
  auto bail = [&](int rc) { ibl_ib_destroy(h); return rc; };
  int rc;
  const size_t inbox = (size_t)g->n_e * h->ldb;
  if ((rc = dalloc(&h->cin, inbox)) || (rc = dalloc(&h->vin, inbox)) || (rc = dalloc(&h->ch8, (size_t)g->n_v * h->ldb)) ||
      (rc = dalloc(&h->flags, (size_t)imax * kShards)) || (rc = dalloc(&h->dL, 1)))
    return bail(rc);
  if (hipMemset(h->cin, 0, inbox) != hipSuccess || hipMemset(h->vin, 0, inbox) != hipSuccess ||
      hipMemset(h->ch8, 0, (size_t)g->n_v * h->ldb) != hipSuccess || hipMemset(h->flags, 0, sizeof(int32_t) * imax * kShards) != hipSuccess)
    return bail(fail(IBL_EHIP, "hipMemset failed"));

  const std::vector<int> cdeg = present(g->h_cn_deg), vdeg = present(g->h_vn_deg);
  const bool deg_ok = CM <= kMaxD && VM <= kMaxD;
  const int cn_nraw = h->match ? CM - 3 : CM - 2;
  int cn_nt = cn_nraw, vn_nraw = h->match ? std::max(VM - 2, 0) : VM - 1, vn_nt = vn_nraw;
  if (h->match) {
    cn_nt += (int)cdeg.size();
    for (int d : vdeg) vn_nt += (d >= 2);
  }
  const int max_nt = (kLdsBytes / kSuper) * 8;   // whole super-regions of 2 quads: 16 tables
  // table slot of each column-fetched input (cn_ncols / vn_ncols): raw fold table, or the degree's
  // final (matching-composed) table; slots are numbered as in the pass images below
  std::vector<int> ccol_slot, vcol_slot;   // column image index -> table slot
  auto col_index = [](std::vector<int>& v, int s) {
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i] == s) return (int8_t)i;
    v.push_back(s);
    return (int8_t)(v.size() - 1);
  };
  {
    int slot = cn_nraw;
    for (int d : cdeg) {
      const int fs = h->match ? slot++ : (d >= 3 ? d - 3 : 0);
      for (int i = 0, nc = cn_ncols(d); i < nc; ++i) {
        const int l = d - nc + i - 2;   // input j = d-nc+i meets table j-2 in every non-prefix chain
        h->cn_ccol[d][i] = col_index(ccol_slot, l == d - 3 ? fs : l);
      }
    }
    slot = vn_nraw;
    for (int d : vdeg) {
      if (d < 2) continue;
      const int fs = h->match ? slot++ : d - 2;
      for (int i = 0, nc = vn_ncols(d); i < nc; ++i) {
        const int l = d - nc + i - 1;   // input j meets table j-1
        h->vn_ccol[d][i] = col_index(vcol_slot, l == d - 2 ? fs : l);
      }
    }
  }
  h->cn_ncs = (int)ccol_slot.size();
  h->vn_ncs = (int)vcol_slot.size();
  const bool lds_ok = fast_lds(cn_nt, h->cn_ncs) <= (size_t)kLdsBytes && fast_lds(std::max(vn_nt, 1), h->vn_ncs) <= (size_t)kLdsBytes;
  h->fast = !(flags & IBL_FLAG_FORCE_GENERIC) && Tc == T && T <= kTP && deg_ok && cn_nt <= max_nt &&
            vn_nt <= max_nt && VM <= max_nt && cn_nt > 0 && lds_ok;

  if (h->fast) {
    // ---------------- CN images: pass p = 0 (iteration 0 ops) .. imax-1
    std::vector<uint32_t> cimg, vimg, dimg, ccimg, vcimg;
    const int64_t T2 = (int64_t)T * T;
    auto cn_raw = [&](int p, int l, int t, int m) -> int {
      int64_t idx;
      if (p == 0) idx = (l == 0) ? (int64_t)t * Tc + m : (int64_t)Tc * Tc + (int64_t)(l - 1) * Tc * T + (int64_t)t * T + m;
      else idx = (int64_t)Tc * Tc + (int64_t)(CM - 3) * Tc * T + (int64_t)(p - 1) * (CM - 2) * T2 + l * T2 + (int64_t)t * T + m;
      return cn_lut[idx];
    };
    auto vn_raw = [&](int k, int l, int t, int m) -> int {
      const int64_t off = (int64_t)k * ((int64_t)Tc * T + (int64_t)(VM - 1) * T2);
      const int64_t idx = off + (l == 0 ? (int64_t)t * T + m : (int64_t)Tc * T + (int64_t)(l - 1) * T2 + (int64_t)t * T + m);
      return vn_lut[idx];
    };
    for (int p = 0; p < imax; ++p) {
      std::vector<Table> tbs;
      for (int l = 0; l < cn_nraw; ++l) tbs.push_back(make_table(T, [&](int t, int m) { return cn_raw(p, l, t, m); }));
      int slot = cn_nraw;
      for (int d : cdeg) {
        if (!h->match) {
          h->cn_fslot[d] = d >= 3 ? d - 3 : 0;
          continue;
        }
        const int64_t mrow = (int64_t)p * T * CM + (int64_t)(d - 1) * T;
        if (d == 2) tbs.push_back(make_table(T, [&](int t, int) { return match_cn[mrow + t]; }));
        else tbs.push_back(make_table(T, [&](int t, int m) { return match_cn[mrow + cn_raw(p, d - 3, t, m)]; }));
        h->cn_fslot[d] = slot++;
      }
      append_pass(cimg, tbs, regions_of(cn_nt));
      append_cols(ccimg, tbs, ccol_slot);
    }
    h->cn_nt = regions_of(cn_nt);
    // ---------------- VN images: pass k = 0 .. imax-2 (extrinsic), decision images k = 0 .. imax-1
    for (int k = 0; k < std::max(imax - 1, 1); ++k) {
      std::vector<Table> tbs;
      for (int l = 0; l < vn_nraw; ++l) tbs.push_back(make_table(T, [&](int t, int m) { return vn_raw(k, l, t, m); }));
      int slot = vn_nraw;
      for (int d : vdeg) {
        if (d < 2) continue;
        if (!h->match) {
          h->vn_fslot[d] = d - 2;
          continue;
        }
        const int64_t mrow = (int64_t)k * T * VM + (int64_t)(d - 1) * T;
        tbs.push_back(make_table(T, [&](int t, int m) { return match_vn[mrow + vn_raw(k, d - 2, t, m)]; }));
        h->vn_fslot[d] = slot++;
      }
      append_pass(vimg, tbs, regions_of(std::max(vn_nt, 1)));
      append_cols(vcimg, tbs, vcol_slot);
    }
    h->vn_nt = regions_of(std::max(vn_nt, 1));
    for (int k = 0; k < imax; ++k) {
      std::vector<Table> tbs;
      for (int l = 0; l < VM; ++l) tbs.push_back(make_table(T, [&](int t, int m) { return vn_raw(k, l, t, m); }));
      append_pass(dimg, tbs, regions_of(VM));
    }
    h->dec_nt = regions_of(VM);
    if ((rc = dupload(&h->cn_img, cimg.data(), cimg.size())) || (rc = dupload(&h->vn_img, vimg.data(), vimg.size())) ||
        (rc = dupload(&h->dec_img, dimg.data(), dimg.size())) ||
        (rc = dupload(&h->cn_cimg, ccimg.data(), ccimg.size())) || (rc = dupload(&h->vn_cimg, vcimg.data(), vcimg.size())))
      return bail(rc);
    if ((rc = pick_cfg(0, CM, 4 * h->cn_nt, h->cn_ncs, g->num_cus, &h->kcn)) ||
        (rc = pick_cfg(1, VM, 4 * h->vn_nt, h->vn_ncs, g->num_cus, &h->kvn)) ||
        (rc = pick_cfg(2, VM, 4 * h->dec_nt, 0, g->num_cus, &h->kdec)))
      return bail(rc);
    // The fast kernels are built to run without a private segment (launch bounds sized to the node
    // bodies' registers, item buffers forced inline). A build whose compiler spills registers or passes
    // an item through scratch would silently lose the register budget the design rests on, and such a
    // build once faulted (DESIGN.md "Private segment"): refuse it loudly instead.
    size_t priv = 0;
    const char* kname = "";
    HIPCHK(ib_fast_private_bytes(CM, VM, &priv, &kname));
#if IBL_DIAG
    const bool allow_scratch = getenv("IBL_ALLOW_SCRATCH") != nullptr;   // diagnostic builds: the spill experiment
#else
    const bool allow_scratch = false;
#endif
    if (priv != 0 && !allow_scratch)
      return bail(fail(IBL_EHIP, std::string("fast-path kernel ") + kname + " has a " + std::to_string(priv) +
                                     "-byte private segment (register spill / scratch item): rebuild required"));
    if ((rc = ib_fused_setup(h))) return bail(rc);
    // small-batch per-pass kernels: the fast path's tables without column images; used for B <= small_b
    // (IBL_SMALL_B at create overrides the default, 0 turns them off)
    if (h->cn_ncs == 0 && h->vn_ncs == 0) {
      HIPCHK(ib_small_private_bytes(CM, VM, &priv, &kname));
      const char* sb = getenv("IBL_SMALL_B");
      h->s_ok = priv == 0;
      h->small_b = h->s_ok ? (sb ? std::max(0, atoi(sb)) : kSmallBatchDefault) : 0;
      const char* sg = getenv("IBL_SMALL_GRAPH");
      h->s_graphs.on = !(sg && sg[0] == '0');
      h->s_lds_cn = lds_of_quads(h->cn_nt);
      h->s_lds_vn = lds_of_quads(h->vn_nt);
      h->s_lds_dec = lds_of_quads(h->dec_nt);
    }
  } else {
    h->cn_len = cn_len; h->vn_len = vn_len;
    if ((rc = dupload(&h->cn_lut, cn_lut, cn_len)) || (rc = dupload(&h->vn_lut, vn_lut, vn_len))) return bail(rc);
    if (h->match) {
      h->mc_len = mc_len; h->mv_len = mv_len;
      if ((rc = dupload(&h->mc, match_cn, mc_len)) || (rc = dupload(&h->mv, match_vn, mv_len))) return bail(rc);
    }
  }
  *out = h;
  return IBL_OK;
}

int ibl_ib_path(const ibl_ib* h) { return h && h->fast ? 1 : 0; }

int ibl_ib_set_small_batch(ibl_ib* h, int32_t max_b) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (max_b < 0) return fail(IBL_EINVAL, "max_b must be >= 0");
  if (max_b > 0 && !(h->fast && h->cn_ncs == 0 && h->vn_ncs == 0 && h->s_lds_cn > 0))
    return fail(IBL_EUNSUPPORTED, "the small-batch kernels need the fast path (T_ch = T_dec <= 16, degrees <= 16)");
  if (max_b > 0 && !h->s_ok)   // create turned them off: this build's small-batch kernels need scratch
    return fail(IBL_EUNSUPPORTED, "the small-batch kernels of this build have a private segment: rebuild required");
  h->small_b = max_b;
  return IBL_OK;
}

int ibl_ib_small_batch(const ibl_ib* h, int32_t* max_b) {
  if (!h || !max_b) return fail(IBL_EINVAL, "NULL argument");
  *max_b = h->small_b;
  return IBL_OK;
}


int ibl_ib_set_path(ibl_ib* h, int32_t path) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (path != IBL_PATH_AUTO && path != IBL_PATH_PASSES && path != IBL_PATH_FUSED)
    return fail(IBL_EINVAL, "path must be IBL_PATH_AUTO, IBL_PATH_PASSES or IBL_PATH_FUSED");
  if (path == IBL_PATH_FUSED && !h->fused_ok)
    return fail(IBL_EUNSUPPORTED, "code does not fit the fused IB kernel (fast path, E * 4 B of messages plus the "
                                  "largest pass's tables within 160 KiB, check degrees >= 2)");
  h->path = path;
  return IBL_OK;
}

int ibl_ib_fused_ncw(const ibl_ib* h, int32_t B, int32_t* ncw) {
  if (!h || !ncw) return fail(IBL_EINVAL, "NULL argument");
  if (B < 1 || B > h->max_batch) return fail(IBL_EINVAL, "B must lie in [1, max_batch]");
  *ncw = ib_fused_in_use(h) ? ib_fused_ncw(h, B) : 0;
  return IBL_OK;
}

int ibl_ib_path_in_use(const ibl_ib* h, int32_t* fused) {
  if (!h || !fused) return fail(IBL_EINVAL, "NULL argument");
  *fused = ib_fused_in_use(h) ? 1 : 0;
  return IBL_OK;
}

int ibl_ib_timing(ibl_ib* h, int32_t enable) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  h->timer.on = enable != 0;
  return IBL_OK;
}
int ibl_ib_timing_read(ibl_ib* h, double* cn_ms, int32_t* cn_n, double* vn_ms, int32_t* vn_n) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  return h->timer.read(cn_ms, cn_n, vn_ms, vn_n) ? fail(IBL_EHIP, "event timing failed") : IBL_OK;
}
int ibl_float_timing(ibl_float* h, int32_t enable) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  h->timer.on = enable != 0;
  return IBL_OK;
}
int ibl_float_timing_read(ibl_float* h, double* cn_ms, int32_t* cn_n, double* vn_ms, int32_t* vn_n) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  return h->timer.read(cn_ms, cn_n, vn_ms, vn_n) ? fail(IBL_EHIP, "event timing failed") : IBL_OK;
}

void ibl_ib_destroy(ibl_ib* h) {
  if (!h) return;
  (void)hipSetDevice(h->g->device);
  dfree(h->cin); dfree(h->vin); dfree(h->ch8); dfree(h->flags); dfree(h->dL);
  dfree(h->cn_img); dfree(h->vn_img); dfree(h->dec_img); dfree(h->cn_cimg); dfree(h->vn_cimg);
  dfree(h->cn_lut); dfree(h->vn_lut); dfree(h->mc); dfree(h->mv);
  dfree(h->f_cn_task); dfree(h->f_vn_task); dfree(h->f_vn_node); dfree(h->f_vn_slot);
  delete h;
}

int ibl_ib_decode(ibl_ib* h, const void* d_ch, int32_t ch_dtype, int32_t B, void* d_out, int32_t out_dtype,
                  int32_t early_stop, int32_t* d_iters, void* stream) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (B < 1 || B > h->max_batch) return fail(IBL_EINVAL, "B must lie in [1, max_batch]");
  if (ch_dtype != kU8 && ch_dtype != kI32) return fail(IBL_EINVAL, "channel dtype must be IBL_U8 or IBL_I32");
  if (out_dtype != kU8 && out_dtype != kI32) return fail(IBL_EINVAL, "output dtype must be IBL_U8 or IBL_I32");
  if (!d_ch || !d_out) return fail(IBL_EINVAL, "NULL buffer");
  const ibl_graph* g = h->g;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(g->device));
  const int I = h->imax;
  const bool early = early_stop != 0 && I > 1;
  if (early) HIPCHK(hipMemsetAsync(h->flags, 0, sizeof(int32_t) * (size_t)I * kShards, s));
  if (ib_fused_in_use(h)) {
    // channel as [group][N] dwords of 8 nibbles (the fused kernel's layout), in the staging buffer
    uint32_t* chT = reinterpret_cast<uint32_t*>(h->ch8);
    HIPCHK(launch_ib_stage_t(d_ch, ch_dtype, g->n_v, B, h->f_vn_node, chT, s));
    IbFusedArgs f{};
    f.cn_img = h->cn_img; f.vn_img = h->vn_img; f.dec_img = h->dec_img; f.chT = chT;
    f.cn_task = h->f_cn_task; f.vn_task = h->f_vn_task; f.vn_node = h->f_vn_node; f.vn_slot = h->f_vn_slot;
    f.out = d_out; f.unsat = early ? h->flags : nullptr; f.dL = nullptr;
    std::memcpy(f.cn_fslot, h->cn_fslot, sizeof(f.cn_fslot));
    std::memcpy(f.vn_fslot, h->vn_fslot, sizeof(f.vn_fslot));
    f.cn_nt = h->cn_nt; f.vn_nt = h->vn_nt; f.dec_nt = h->dec_nt; f.nreg = h->f_nreg; f.dbuf = h->f_dbuf;
    f.n_cn_nodes = g->n_c; f.cn_uni = h->f_cn_uni; f.vn_uni = h->f_vn_uni;
    f.n_e = (int32_t)g->n_e; f.n_v = g->n_v; f.n_cn_tasks = h->f_ncn; f.n_vn_tasks = h->f_nvn;
    f.B = B; f.imax = I; f.half = h->T / 2; f.match = h->match; f.out_dtype = out_dtype;
    const size_t esz = out_dtype == kU8 ? 1 : 4;
    f.aligned = ((B % 4) == 0 && ((uintptr_t)d_out % (4 * esz)) == 0) ? 1 : 0;
    f.ngroups = (B + 7) / 8;
    f.ncw = ib_fused_ncw(h, B);
    const int grid = std::min(h->f_grid, f.ngroups * (8 / f.ncw));
#if IBL_DIAG
    // diagnostic builds only: IBL_TRACE_FUSED=<file> records block 0's clock at every phase boundary of its
    // first group (with -DIBL_FUSED_TRACE=1 kernels, tools/variants.py ftrace)
    const char* ftrace = getenv("IBL_TRACE_FUSED");
    const size_t ntr = (size_t)3 * (2 * I + 4);
    if (ftrace) {
      HIPCHK(hipMalloc((void**)&f.trace, sizeof(uint64_t) * ntr));
      HIPCHK(hipMemsetAsync(f.trace, 0, sizeof(uint64_t) * ntr, s));
    }
#endif
    HIPCHK(h->timer.timed(0, s, [&] { return launch_ib_fused(f, h->CM, h->VM, grid, h->f_block, h->f_lds, s); }));
#if IBL_DIAG
    if (ftrace) {
      std::vector<uint64_t> hv(ntr);
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipMemcpy(hv.data(), f.trace, sizeof(uint64_t) * ntr, hipMemcpyDeviceToHost));
      (void)hipFree(f.trace);
      f.trace = nullptr;
      if (FILE* fp = fopen(ftrace, "wb")) {
        fwrite(hv.data(), sizeof(uint64_t), ntr, fp);
        fclose(fp);
      }
    }
#endif
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    if (early) {   // pass 2: re-run the batch to the stop iteration (a no-op when it is imax-1)
      f.unsat = nullptr;
      f.dL = h->dL;
      HIPCHK(h->timer.timed(0, s, [&] { return launch_ib_fused(f, h->CM, h->VM, grid, h->f_block, h->f_lds, s); }));
    }
    return IBL_OK;
  }
  if (h->fast && B <= h->small_b) {
    // small batch: (task, word) items, lane = node (ib_*_small); the pass schedule of the fast path.
    // Rows are packed to the batch's words (4 * nwords bytes, not the per-pass path's ldb / 2): a pass
    // then touches E * 4 * nwords bytes of each inbox (B = 2 on DVB-S2: 0.9 MB, resident in the L2s and
    // the MALL) instead of one 128-B line per edge (29 MB)
    const int nwords = (B + 7) / 8, ldbb = 4 * nwords;
    HIPCHK(launch_ib_stage4(d_ch, ch_dtype, g->n_v, B, h->ch8, ldbb, s));
    auto grid_of = [&](int ntask, size_t lds) {
      const int per_cu = std::max(1, (int)(kLdsBytes / std::max<size_t>(lds, 1)));
      const int wpb = small_block(nwords) / 64;
      const int need = (ntask * nwords + wpb - 1) / wpb;
      return std::max(1, std::min(need, per_cu * g->num_cus));
    };
    IbFastArgs cn{}, vn{};
    cn.ch8 = vn.ch8 = h->ch8;
    cn.info = g->cn_info; cn.task = g->cn_task; cn.n_tasks = g->n_cn_task; cn.tgt = g->tgt_cn; cn.out = h->vin;
    vn.info = g->vn_info; vn.task = g->vn_task; vn.n_tasks = g->n_vn_task; vn.tgt = g->tgt_vn; vn.out = h->cin;
    vn.in = h->vin;
    cn.n_nodes = g->n_c; vn.n_nodes = g->n_v;
    cn.nwords = vn.nwords = nwords;
    cn.ldb = vn.ldb = ldbb;
    cn.B = vn.B = B;
    cn.half = vn.half = h->T / 2;
    cn.match = vn.match = h->match;
    cn.nt = h->cn_nt; vn.nt = h->vn_nt;
    std::memcpy(cn.fslot, h->cn_fslot, sizeof(cn.fslot));
    std::memcpy(vn.fslot, h->vn_fslot, sizeof(vn.fslot));
    const int gcn = grid_of(g->n_cn_task, h->s_lds_cn), gvn = grid_of(g->n_vn_task, h->s_lds_vn);
    // the pass chain (decoder buffers only): CN pass 0 from the staged channel, then {VN j, CN j}
    auto chain = [&](hipStream_t st) -> hipError_t {
      IbFastArgs c0 = cn, v = vn;
      c0.in = nullptr; c0.gather = g->csr_cols; c0.img = h->cn_img; c0.gate = nullptr; c0.unsat = nullptr;
      hipError_t e = h->timer.timed(0, st, [&] { return launch_ib_cn_small(c0, h->CM, gcn, h->s_lds_cn, st); });
      if (e != hipSuccess) return e;
      IbFastArgs c = c0;
      c.gather = nullptr;
      c.in = h->cin;
      for (int j = 1; j < I; ++j) {
        const int32_t* gate = (early && j >= 2) ? h->flags + (size_t)(j - 1) * kShards : nullptr;
        v.img = h->vn_img + (size_t)(j - 1) * h->vn_nt * 256;
        v.gate = gate;
        if ((e = h->timer.timed(1, st, [&] { return launch_ib_vn_small(v, h->VM, gvn, h->s_lds_vn, st); })) != hipSuccess)
          return e;
        c.img = h->cn_img + (size_t)j * h->cn_nt * 256;
        c.gate = gate;
        c.unsat = early ? h->flags + (size_t)j * kShards : nullptr;
        if ((e = h->timer.timed(0, st, [&] { return launch_ib_cn_small(c, h->CM, gcn, h->s_lds_cn, st); })) != hipSuccess)
          return e;
      }
      return hipSuccess;
    };
    // replayed from a captured graph, unless per-launch timing is on (bench roofline) or graphs are off
    if (h->s_graphs.on && !h->timer.on) HIPCHK(h->s_graphs.run(B, early ? 1 : 0, s, chain));
    else HIPCHK(chain(s));
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    IbDecArgs dc{};
    dc.vin = h->vin; dc.ch8 = h->ch8; dc.img = h->dec_img; dc.iters = h->dL; dc.out = d_out; dc.out_dtype = out_dtype;
    dc.nt = h->dec_nt; dc.n_nodes = g->n_v; dc.ldb = ldbb; dc.B = B;
    dc.info = g->vn_info; dc.task = g->vn_task; dc.n_tasks = g->n_vn_task; dc.nwords = nwords;
    const size_t esz = out_dtype == kU8 ? 1 : 4;
    dc.aligned = ((B % 4) == 0 && ((uintptr_t)d_out % (4 * esz)) == 0) ? 1 : 0;
    HIPCHK(launch_ib_dec_small(dc, grid_of(g->n_vn_task, h->s_lds_dec), h->s_lds_dec, s));
    return IBL_OK;
  }
  if (h->fast) {
    const int ccn = ib_fast_chunk(h->CM), cvn = ib_fast_chunk(h->VM);
    const int ldbb = h->ldb / 2;
    HIPCHK(launch_ib_stage4(d_ch, ch_dtype, g->n_v, B, h->ch8, ldbb, s));
    IbFastArgs cn{}, vn{};
    cn.ch8 = vn.ch8 = h->ch8;
    cn.info = g->cn_info; cn.tgt = g->tgt_cn; cn.out = h->vin;
    vn.info = g->vn_info; vn.tgt = g->tgt_vn; vn.out = h->cin; vn.in = h->vin;
    cn.n_nodes = g->n_c; vn.n_nodes = g->n_v;
    cn.n_heavy = g->cn_heavy; vn.n_heavy = g->vn_heavy;
#if IBL_DIAG
    // diagnostic builds only (timing, outputs are not decodes): IBL_VN_PART=heavy / light runs the variable
    // pass over one item class only (the degree > kLightD items, or the rest)
    if (const char* vp = getenv("IBL_VN_PART")) {
      if (vp[0] == 'h') {
        vn.n_nodes = g->vn_heavy;
      } else if (vp[0] == 'l') {
        vn.info = g->vn_info + 4 * (size_t)g->vn_heavy;
        vn.n_nodes = g->n_v - g->vn_heavy;
        vn.n_heavy = 0;
      }
    }
#endif
    cn.nchunks = (B + ccn - 1) / ccn;
    vn.nchunks = (B + cvn - 1) / cvn;
    cn.ldb = vn.ldb = ldbb;
    cn.B = vn.B = B;
    cn.half = vn.half = h->T / 2;
    cn.match = vn.match = h->match;
    cn.nt = h->cn_nt; vn.nt = h->vn_nt;
    std::memcpy(cn.fslot, h->cn_fslot, sizeof(cn.fslot));
    std::memcpy(vn.fslot, h->vn_fslot, sizeof(vn.fslot));
    std::memcpy(cn.ccol, h->cn_ccol, sizeof(cn.ccol));
    std::memcpy(vn.ccol, h->vn_ccol, sizeof(vn.ccol));
    cn.ncs = h->cn_ncs; vn.ncs = h->vn_ncs;
    // pass 0: send + checknode_update_iter0, inputs gathered from the staged channel rows
    cn.in = nullptr; cn.gather = g->csr_cols; cn.img = h->cn_img; cn.gate = nullptr; cn.unsat = nullptr;
    cn.cimg = h->cn_cimg;
    auto launch_cn = [&]() { return launch_ib_cn_fast(cn, h->CM, h->kcn.grid, h->kcn.block, h->kcn.lds, s); };
    HIPCHK(h->timer.timed(0, s, launch_cn));
    cn.gather = nullptr;
    uint64_t* trace = nullptr;
#if IBL_DIAG
    // diagnostic builds only: IBL_TRACE_WAVES=<prefix> records {start, end, items|cu} of every wave of the
    // middle iteration's VN and CN launches into <prefix>_vn.bin / <prefix>_cn.bin (uint64 triples)
    const char* trace_path = getenv("IBL_TRACE_WAVES");
    const size_t nwv = (size_t)h->kvn.grid * (h->kvn.block / 64), nwc = (size_t)h->kcn.grid * (h->kcn.block / 64);
    if (trace_path && I > 1) HIPCHK(hipMalloc((void**)&trace, sizeof(uint64_t) * 3 * (nwv + nwc)));
#else
    const size_t nwv = 0;
#endif
    for (int j = 1; j < I; ++j) {
      const int32_t* gate = (early && j >= 2) ? h->flags + (size_t)(j - 1) * kShards : nullptr;
      vn.img = h->vn_img + (size_t)(j - 1) * h->vn_nt * 256;
      vn.cimg = h->vn_cimg + (size_t)(j - 1) * h->vn_ncs * 32;
      vn.gate = gate;
      vn.trace = (trace && j == I / 2) ? trace : nullptr;
      HIPCHK(h->timer.timed(1, s, [&] { return launch_ib_vn_fast(vn, h->VM, h->kvn.grid, h->kvn.block, h->kvn.lds, s); }));
      cn.img = h->cn_img + (size_t)j * h->cn_nt * 256;
      cn.cimg = h->cn_cimg + (size_t)j * h->cn_ncs * 32;
      cn.gate = gate;
      cn.unsat = early ? h->flags + (size_t)j * kShards : nullptr;
      cn.trace = (trace && j == I / 2) ? trace + 3 * nwv : nullptr;
      cn.in = h->cin;
      HIPCHK(h->timer.timed(0, s, launch_cn));
    }
#if IBL_DIAG
    if (trace) {
      std::vector<uint64_t> hv(3 * (nwv + nwc));
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipMemcpy(hv.data(), trace, sizeof(uint64_t) * hv.size(), hipMemcpyDeviceToHost));
      (void)hipFree(trace);
      for (int k = 0; k < 2; ++k) {
        const std::string p = std::string(trace_path) + (k == 0 ? "_vn.bin" : "_cn.bin");
        if (FILE* f = fopen(p.c_str(), "wb")) {
          fwrite(hv.data() + (k == 0 ? 0 : 3 * nwv), sizeof(uint64_t), 3 * (k == 0 ? nwv : nwc), f);
          fclose(f);
        }
      }
    }
#endif
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    IbDecArgs dc{};
    dc.vin = h->vin; dc.ch8 = h->ch8; dc.start = g->vn_start; dc.deg = g->vn_deg; dc.img = h->dec_img;
    dc.iters = h->dL; dc.out = d_out; dc.out_dtype = out_dtype; dc.nt = h->dec_nt; dc.n_nodes = g->n_v;
    dc.nchunks = (B + kChunkDec - 1) / kChunkDec; dc.ldb = ldbb; dc.B = B;
    const size_t esz = out_dtype == kU8 ? 1 : 4;
    dc.aligned = ((B % 4) == 0 && ((uintptr_t)d_out % (4 * esz)) == 0) ? 1 : 0;
    HIPCHK(launch_ib_dec_fast(dc, h->kdec.grid, h->kdec.block, h->kdec.lds, s));
  } else {
    HIPCHK(launch_ib_stage(d_ch, ch_dtype, g->n_v, B, h->ch8, h->ldb, s));
    IbGenArgs cn{}, vn{};
    cn.ch8 = vn.ch8 = h->ch8;
    cn.start = g->cn_start; cn.deg = g->cn_deg; cn.tgt = g->tgt_cn; cn.out = h->vin; cn.lut = h->cn_lut;
    cn.lut_len = h->cn_len; cn.mt = h->mc; cn.mt_len = h->mc_len;
    vn.start = g->vn_start; vn.deg = g->vn_deg; vn.tgt = g->tgt_vn; vn.out = h->cin; vn.in = h->vin; vn.lut = h->vn_lut;
    vn.lut_len = h->vn_len; vn.mt = h->mv; vn.mt_len = h->mv_len;
    cn.Tc = vn.Tc = h->Tc; cn.T = vn.T = h->T; cn.CM = vn.CM = h->CM; cn.VM = vn.VM = h->VM;
    cn.match = vn.match = h->match;
    cn.n_nodes = g->n_c; vn.n_nodes = g->n_v;
    cn.ldb = vn.ldb = h->ldb; cn.B = vn.B = B; cn.half = vn.half = h->T / 2;
    cn.pass = 0; cn.in = nullptr; cn.gather = g->csr_cols;
    HIPCHK(h->timer.timed(0, s, [&] { return launch_ib_cn_gen(cn, s); }));
    cn.in = h->cin; cn.gather = nullptr;
    for (int j = 1; j < I; ++j) {
      const int32_t* gate = (early && j >= 2) ? h->flags + (size_t)(j - 1) * kShards : nullptr;
      vn.pass = j - 1; vn.gate = gate;
      HIPCHK(h->timer.timed(1, s, [&] { return launch_ib_vn_gen(vn, s); }));
      cn.pass = j; cn.gate = gate; cn.unsat = early ? h->flags + (size_t)j * kShards : nullptr;
      HIPCHK(h->timer.timed(0, s, [&] { return launch_ib_cn_gen(cn, s); }));
    }
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    IbGenDecArgs dc{};
    dc.vin = h->vin; dc.ch8 = h->ch8; dc.start = g->vn_start; dc.deg = g->vn_deg; dc.lut = h->vn_lut;
    dc.lut_len = h->vn_len; dc.iters = h->dL; dc.out = d_out; dc.out_dtype = out_dtype; dc.Tc = h->Tc; dc.T = h->T;
    dc.VM = h->VM; dc.n_nodes = g->n_v; dc.ldb = h->ldb; dc.B = B;
    HIPCHK(launch_ib_dec_gen(dc, s));
  }
  return IBL_OK;
}

// ------------------------------------------------------------------ float decoder
}  // extern "C"

namespace {

// candidates the fused kernels' bank-order greedy scans per lane (IBL_FUSED_VWIN at create, A/B; default 256)
size_t fused_vwin() {
  const char* vw = getenv("IBL_FUSED_VWIN");
  return (size_t)std::max(1, vw ? atoi(vw) : 256);
}
int upload_fused_tasks(const FusedTasks& ft, int32_t** cn_task, int32_t** vn_task, int32_t** vn_node, int32_t** vn_slot) {
  int rc;
  if ((rc = dupload(cn_task, ft.cn_task.data(), ft.cn_task.size())) || (rc = dupload(vn_task, ft.vn_task.data(), ft.vn_task.size())) ||
      (rc = dupload(vn_node, ft.vn_node.data(), ft.vn_node.size())) || (rc = dupload(vn_slot, ft.vn_slot.data(), ft.vn_slot.size())))
    return rc;
  return IBL_OK;
}
// Task tables of the fused float kernel (FlFusedArgs). Check nodes sorted by degree (heaviest first,
// stable) and cut into tasks of up to 64 nodes of one degree; edge k of lane i of a check task gets
// slot first + k*count + i. Variable nodes likewise; vn_slot maps each variable edge (task-major,
// k*count + i) to the slot of the same edge. Leaves fused_ok false when the code does not fit.
int fused_setup(ibl_float* h) {
  const ibl_graph* g = h->g;
  const int64_t E = g->n_e;
  int min_dc = 1 << 30;
  for (int32_t d : g->h_cn_deg) min_dc = std::min(min_dc, d);
  if (E >= 65536 || min_dc < 2 || E == 0 || (size_t)(E + g->n_v) * 16 > (size_t)kLdsBytes) return IBL_OK;
  FusedTasks ft;
  int rc;
  // 16-byte slots (ds_read_b128 / ds_write_b128): the natural order (stable by degree) keeps a quasi-cyclic
  // code's lanes on runs of consecutive slots, which conflict less than the dword-bank greedy order;
  // IBL_FUSED_VORDER=1 selects the greedy order (A/B)
  const char* voe = getenv("IBL_FUSED_VORDER");
  build_fused_tasks(*g, &ft, voe && voe[0] == '1', fused_vwin());
  pad_vn_slots(&ft);
  // messages and channel (16-byte slots), 4 counter words, the padded u16 indices (codes whose indices do
  // not fit beside the messages take the per-pass path)
  const size_t lds = (size_t)(E + g->n_v) * 16 + 16 + ft.vn_slot.size() * 2;
  if (lds > (size_t)kLdsBytes) return IBL_OK;
  int bpc = 0, block = 0;
  if (fl_fused_occupancy(h->kind, h->prec, g->dcm, g->dvm, lds, &bpc, &block) != hipSuccess || bpc < 1) {
    (void)hipGetLastError();
    return IBL_OK;
  }
  if ((rc = upload_fused_tasks(ft, &h->f_cn_task, &h->f_vn_task, &h->f_vn_node, &h->f_vn_slot))) return rc;
  h->f_ncn = (int32_t)(ft.cn_task.size() / 4);
  h->f_nvn = (int32_t)(ft.vn_task.size() / 4);
  h->f_nvs = (int32_t)ft.vn_slot.size();
  h->f_lds = lds;
  h->f_grid = bpc * g->num_cus;
  h->fused_ok = true;
  return IBL_OK;
}


// Fused IB decoder eligibility (fast path, no column images, messages + the largest pass's table
// quads within the CU's LDS, check degree >= 2, an occupancy of >= 1 block without scratch) and
// task tables. Leaves fused_ok false when the code does not fit.
int ib_fused_setup(ibl_ib* h) {
  const ibl_graph* g = h->g;
  if (!h->fast || h->cn_ncs || h->vn_ncs || g->n_e == 0) return IBL_OK;
  int min_dc = 1 << 30;
  for (int32_t d : g->h_cn_deg) min_dc = std::min(min_dc, d);
  if (min_dc < 2) return IBL_OK;
  const int nreg = std::max(h->cn_nt, std::max(h->vn_nt, h->dec_nt));
  // one table set: tables, raw images, slots; two sets (see TablePrefetch; a single quad's two sets share
  // one super-region) where they fit beside the slots; IBL_FUSED_DBUF=0 turns them off (A/B)
  const size_t lds1 = lds_of_quads(nreg) + (size_t)nreg * 1024 + (size_t)g->n_e * 4 + 16;
  const size_t lds2 = lds_of_quads(2 * nreg) + (size_t)g->n_e * 4 + 16;
  const char* dbe = getenv("IBL_FUSED_DBUF");
  const bool dbuf = nreg <= 2 && lds2 <= (size_t)kLdsBytes && !(dbe && dbe[0] == '0');   // set offset: ib_fused
  const size_t lds = dbuf ? lds2 : lds1;
  if (lds > (size_t)kLdsBytes) return IBL_OK;
  int bpc = 0, block = 0;
  size_t priv = 0;
  if (ib_fused_occupancy(h->CM, h->VM, 8, lds, &bpc, &block, &priv) != hipSuccess || bpc < 1 || priv != 0) {
    (void)hipGetLastError();
    return IBL_OK;
  }
  {   // the half-group instantiation (4 codewords per workgroup, small batches) under the same bounds
    int bpc4 = 0, block4 = 0;
    size_t priv4 = 0;
    h->f_half_ok = ib_fused_occupancy(h->CM, h->VM, 4, lds, &bpc4, &block4, &priv4) == hipSuccess && bpc4 == bpc &&
                   block4 == block && priv4 == 0;
    (void)hipGetLastError();
  }
  FusedTasks ft;
  int rc;
  const char* voe = getenv("IBL_FUSED_VORDER");
  build_fused_tasks(*g, &ft, !(voe && voe[0] == '0'), fused_vwin());
  if ((rc = upload_fused_tasks(ft, &h->f_cn_task, &h->f_vn_task, &h->f_vn_node, &h->f_vn_slot))) return rc;
  h->f_ncn = (int32_t)(ft.cn_task.size() / 4);
  h->f_nvn = (int32_t)(ft.vn_task.size() / 4);
  // single-degree sides: task records follow from the task index (IbFusedArgs::cn_uni / vn_uni);
  // IBL_FUSED_UNIFORM=0 keeps the loaded records (A/B)
  const char* une = getenv("IBL_FUSED_UNIFORM");
  if (!(une && une[0] == '0')) {
    auto uniform = [](const std::vector<int32_t>& task, int32_t n, bool vn) {
      if (task.empty()) return 0;
      const int32_t d = task[2];
      for (size_t t = 0; t < task.size() / 4; ++t) {
        const int32_t p = (int32_t)(64 * t), cnt = std::min<int32_t>(64, n - p);
        const int32_t* r = &task[4 * t];
        if (r[1] != cnt || r[2] != d || (vn ? (r[0] != p || r[3] != p * d) : r[0] != p * d)) return 0;
      }
      return (int)d;
    };
    h->f_cn_uni = uniform(ft.cn_task, g->n_c, false);
    h->f_vn_uni = uniform(ft.vn_task, g->n_v, true);
  }
  if (const char* ne = getenv("IBL_FUSED_NCW")) h->f_ncw_forced = atoi(ne);
  h->f_nreg = nreg;
  h->f_dbuf = dbuf ? 1 : 0;
  h->f_lds = lds;
  h->f_block = block;
  h->f_grid = bpc * g->num_cus;
  h->fused_ok = true;
  return IBL_OK;
}

bool ib_fused_in_use(const ibl_ib* h) { return h->fused_ok && h->path != IBL_PATH_PASSES; }

// The fold's device state (second check inbox, per-check records, unfolded variable list) once a batch can reach
// the per-pass kernels (max_batch > small_b): decoders that only ever run the small-batch kernels — the
// reference's DVB-S2 driver decodes msg_at_time = 2 — do not hold a fourth E x ldb inbox.
int fold_alloc(ibl_float* h) {
  if (h->n_folded == 0 || h->cin2 || h->max_batch <= h->small_b) return IBL_OK;
  const size_t inbox = (size_t)h->g->n_e * h->ldb * (h->prec == kF32 ? 4 : 8);
  uint8_t* c2 = nullptr;
  int rc = dalloc(&c2, inbox);
  if (rc) return rc;
  if (hipMemset(c2, 0, inbox) != hipSuccess) {
    dfree(c2);
    return fail(IBL_EHIP, "hipMemset failed");
  }
  if ((rc = dupload(&h->fold, h->fold_rec.data(), h->fold_rec.size())) ||
      (rc = dupload(&h->vn_nodes, h->fold_rest.data(), h->fold_rest.size()))) {
    dfree(c2); dfree(h->fold); dfree(h->vn_nodes);
    h->fold = h->vn_nodes = nullptr;
    return rc;
  }
  h->cin2 = c2;
  return IBL_OK;
}
}  // namespace

extern "C" {

int ibl_float_set_path(ibl_float* h, int32_t path) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (path != IBL_PATH_AUTO && path != IBL_PATH_PASSES && path != IBL_PATH_FUSED)
    return fail(IBL_EINVAL, "path must be IBL_PATH_AUTO, IBL_PATH_PASSES or IBL_PATH_FUSED");
  if (path == IBL_PATH_FUSED && !h->fused_ok)
    return fail(IBL_EUNSUPPORTED, "code does not fit the fused kernel ((E + N) * 16 B > 160 KiB or a check degree < 2)");
  h->path = path;
  return IBL_OK;
}

int ibl_float_set_small_batch(ibl_float* h, int32_t max_b) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (max_b < 0) return fail(IBL_EINVAL, "max_b must be >= 0");
  if (max_b > 0 && !h->s_ok)   // create turned them off: this build's small-batch kernels need scratch
    return fail(IBL_EUNSUPPORTED, "the small-batch kernels of this build have a private segment: rebuild required");
  HIPCHK(hipSetDevice(h->g->device));
  const int32_t old = h->small_b;
  h->small_b = max_b;
  int rc = fold_alloc(h);   // batches above the new threshold take the per-pass kernels, which fold
  if (rc) h->small_b = old;
  return rc;
}

int ibl_float_small_batch(const ibl_float* h, int32_t* max_b) {
  if (!h || !max_b) return fail(IBL_EINVAL, "NULL argument");
  *max_b = h->small_b;
  return IBL_OK;
}

int ibl_float_folded(const ibl_float* h, int32_t* n_folded) {
  if (!h || !n_folded) return fail(IBL_EINVAL, "NULL argument");
  *n_folded = h->n_folded;
  return IBL_OK;
}

int ibl_float_input_check(ibl_float* h, int32_t* violations, void* stream) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  // The counter belongs to the decoder and collects every decode's staging, on any stream: synchronise the whole
  // device (not only `stream`) so no decode still in flight elsewhere adds to it between the read and the clear.
  (void)stream;
  HIPCHK(hipSetDevice(h->g->device));
  HIPCHK(hipDeviceSynchronize());
  int32_t n = 0;
  HIPCHK(hipMemcpy(&n, h->bad, sizeof(int32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(h->bad, 0, sizeof(int32_t)));
  if (violations) *violations = n;
  if (n > 0)
    return fail(IBL_EINVAL, std::to_string(n) + (h->kind == IBL_BP
                                                     ? (h->prec == kF64 ? " channel LLR(s) NaN or |x| > 709.78 (BP precondition)"
                                                                          : " channel LLR(s) NaN or infinite (BP precondition)")
                                                     : " channel LLR(s) NaN (min-sum precondition)") +
                                ": those decodes' outputs are unspecified");
  return IBL_OK;
}

int ibl_float_path_in_use(const ibl_float* h, int32_t* fused) {
  if (!h || !fused) return fail(IBL_EINVAL, "NULL argument");
  *fused = (h->fused_ok && h->path != IBL_PATH_PASSES) ? 1 : 0;
  return IBL_OK;
}

int ibl_float_create(const ibl_graph* g, int32_t kind, int32_t imax, double llr_max, int32_t precision,
                     int32_t max_batch, ibl_float** out) {
  if (!out) return fail(IBL_EINVAL, "out is NULL");
  *out = nullptr;
  if (!g) return fail(IBL_EINVAL, "graph is NULL");
  if (kind != IBL_MINSUM && kind != IBL_BP) return fail(IBL_EINVAL, "kind must be IBL_MINSUM or IBL_BP");
  if (precision != kF32 && precision != kF64) return fail(IBL_EINVAL, "precision must be IBL_F32 or IBL_F64");
  if (imax < 1 || max_batch < 1) return fail(IBL_EINVAL, "imax and max_batch must be >= 1");
  if (g->dcm > kMaxD || g->dvm > kMaxD) return fail(IBL_EUNSUPPORTED, "float decoders support node degrees <= 16");
  HIPCHK(hipSetDevice(g->device));
  auto* h = new ibl_float();
  h->g = g; h->kind = kind; h->imax = imax; h->prec = precision; h->max_batch = max_batch; h->llr_max = llr_max;
  // rows padded to the widest wave item of the per-pass kernels (fp32 256 / fp64 128 codewords; 512 with IBL_FL_VN2
  // builds), not beyond: the reference's DVB-S2 driver decodes msg_at_time = 2 in fp64
  const int pad = std::max(64 * (precision == kF32 ? 4 : 2), fl_vn_chunk(precision, g->dvm));
  h->ldb = (max_batch + pad - 1) / pad * pad;
  const size_t es = precision == kF32 ? 4 : 8;
  const size_t inbox = (size_t)g->n_e * h->ldb * es;
  int rc;
  auto bail = [&](int r) { ibl_float_destroy(h); return r; };
  uint8_t *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
  if ((rc = dalloc(&a, inbox)) || (rc = dalloc(&b, inbox)) || (rc = dalloc(&c, inbox)) ||
      (rc = dalloc(&d, (size_t)g->n_v * h->ldb * es)) || (rc = dalloc(&h->flags, (size_t)imax * kShards)) ||
      (rc = dalloc(&h->dL, 1)) || (rc = dalloc(&h->bad, 1))) {
    dfree(a); dfree(b); dfree(c); dfree(d);
    return bail(rc);
  }
  h->cin = a; h->vbuf0 = b; h->vbuf1 = c; h->chf = d;
  if (hipMemset(a, 0, inbox) != hipSuccess || hipMemset(b, 0, inbox) != hipSuccess || hipMemset(c, 0, inbox) != hipSuccess ||
      hipMemset(h->bad, 0, sizeof(int32_t)) != hipSuccess)
    return bail(fail(IBL_EHIP, "hipMemset failed"));
  int bpc = 0;
  // at most 16 waves per CU: with a second block per CU its waves issue behind the first block's
  // (oldest-first) and the per-block work counters cannot rebalance across blocks
  if (fl_occupancy(0, kind, precision, g->dcm, &bpc) != hipSuccess || bpc < 1) bpc = 1;
  // (A/B knob, read once here: IBL_FL_WAVES = waves per CU the per-pass grids may fill, default 16)
  const char* fw = getenv("IBL_FL_WAVES");
  const int wcap = std::max(16, fw ? atoi(fw) : 16) * 64;
  h->grid_cn = std::min(bpc, wcap / fl_block(0, kind, precision, g->dcm)) * g->num_cus;
  if (fl_occupancy(1, kind, precision, g->dvm, &bpc) != hipSuccess || bpc < 1) bpc = 1;
  h->grid_vn = std::min(bpc, wcap / fl_block(1, kind, precision, g->dvm)) * g->num_cus;
  if ((rc = fused_setup(h))) return bail(rc);
  {  // degree-2 variable fold of the per-pass path (IBL_FL_FOLD=0 at create turns it off: A/B); its second check
     // inbox is allocated only once some batch can reach the per-pass kernels (max_batch > small_b, fold_alloc)
    const char* fe = getenv("IBL_FL_FOLD");
    if (!(fe && fe[0] == '0') && (h->n_folded = plan_fold(*g, &h->fold_rec, &h->fold_rest)) > 0)
      h->n_vn_nodes = (int32_t)h->fold_rest.size();
    else
      h->n_folded = 0;
  }
  {  // same guard as the IB fast path: the float kernels are built to run without scratch
    size_t priv = 0;
    const char* kname = "";
    HIPCHK(fl_private_bytes(kind, precision, g->dcm, g->dvm, h->fused_ok, &priv, &kname));
    if (priv != 0)
      return bail(fail(IBL_EHIP, std::string("float kernel ") + kname + " has a " + std::to_string(priv) +
                                     "-byte private segment (register spill): rebuild required"));
    // small-batch kernels (IBL_SMALL_B at create overrides the default; off if they would need scratch)
    HIPCHK(fl_small_private_bytes(kind, precision, g->dcm, g->dvm, &priv, &kname));
    const char* sb = getenv("IBL_SMALL_B");
    h->s_ok = priv == 0;
    h->small_b = h->s_ok ? (sb ? std::max(0, atoi(sb)) : kFlSmallBatchDefault) : 0;
    const char* sg = getenv("IBL_SMALL_GRAPH");
    h->s_graphs.on = !(sg && sg[0] == '0');
  }
  if ((rc = fold_alloc(h))) return bail(rc);
  *out = h;
  return IBL_OK;
}

void ibl_float_destroy(ibl_float* h) {
  if (!h) return;
  (void)hipSetDevice(h->g->device);
  dfree(h->cin); dfree(h->vbuf0); dfree(h->vbuf1); dfree(h->chf); dfree(h->flags); dfree(h->dL);
  dfree(h->cin2); dfree(h->fold); dfree(h->vn_nodes); dfree(h->bad);
  dfree(h->f_cn_task); dfree(h->f_vn_task); dfree(h->f_vn_node); dfree(h->f_vn_slot);
  delete h;
}

int ibl_float_decode(ibl_float* h, const void* d_llr, int32_t llr_dtype, int32_t B, void* d_out, int32_t out_dtype,
                     int32_t early_stop, int32_t* d_iters, void* stream) {
  if (!h) return fail(IBL_EINVAL, "decoder is NULL");
  if (B < 1 || B > h->max_batch) return fail(IBL_EINVAL, "B must lie in [1, max_batch]");
  if ((llr_dtype != kF32 && llr_dtype != kF64) || (out_dtype != kF32 && out_dtype != kF64))
    return fail(IBL_EINVAL, "LLR dtypes must be IBL_F32 or IBL_F64");
  if (!d_llr || !d_out) return fail(IBL_EINVAL, "NULL buffer");
  const ibl_graph* g = h->g;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(g->device));
  const int I = h->imax;
  const bool early = early_stop != 0 && I > 1;
  const int cwl = h->prec == kF32 ? 4 : 2;
  const int nchunks = (B + 64 * cwl - 1) / (64 * cwl);
  // the staging kernels count precondition violations (float_kernels.hip llr_bad): min-sum NaN; BP NaN and, for
  // the fp64 decoder, |x| > ln(DBL_MAX), for the fp32 decoder +-inf
  const int rule = h->kind == IBL_BP ? (h->prec == kF64 ? 2 : 3) : 1;
  if (early) HIPCHK(hipMemsetAsync(h->flags, 0, sizeof(int32_t) * (size_t)I * kShards, s));
  if (h->fused_ok && h->path != IBL_PATH_PASSES) {
    HIPCHK(launch_fl_stage_t(d_llr, llr_dtype, g->n_v, B, h->f_vn_node, h->chf, h->prec, rule, h->bad, s));
    FlFusedArgs fa{};
    fa.ch = h->chf; fa.cn_task = h->f_cn_task; fa.vn_task = h->f_vn_task; fa.vn_node = h->f_vn_node;
    fa.vn_slot = h->f_vn_slot; fa.out = d_out; fa.unsat = early ? h->flags : nullptr; fa.dL = nullptr;
    fa.llr_max = h->llr_max; fa.n_e = (int32_t)g->n_e; fa.n_v = g->n_v; fa.n_cn_tasks = h->f_ncn;
    fa.n_vn_tasks = h->f_nvn; fa.n_vs = h->f_nvs; fa.ldb = h->ldb; fa.B = B; fa.imax = I; fa.out_dtype = out_dtype;
    fa.ngroups = (B + cwl - 1) / cwl;
#if IBL_DIAG
    const char* ftrace = getenv("IBL_TRACE_FUSED");   // diagnostic builds: phase clocks of block 0's first group
    const size_t ntr = (size_t)kFlTraceWords * (2 * I + 4);
    if (ftrace) {
      HIPCHK(hipMalloc((void**)&fa.trace, sizeof(uint64_t) * ntr));
      HIPCHK(hipMemsetAsync(fa.trace, 0, sizeof(uint64_t) * ntr, s));
    }
#endif
    const size_t esz = out_dtype == kF32 ? 4 : 8;
    fa.aligned = ((B % cwl) == 0 && ((uintptr_t)d_out % (cwl * esz)) == 0) ? 1 : 0;
    const int grid = std::min(fa.ngroups, h->f_grid);
    HIPCHK(h->timer.timed(0, s, [&] { return launch_fl_fused(fa, h->kind, h->prec, g->dcm, g->dvm, grid, h->f_lds, s); }));
#if IBL_DIAG
    if (ftrace) {
      std::vector<uint64_t> hv(ntr);
      HIPCHK(hipStreamSynchronize(s));
      HIPCHK(hipMemcpy(hv.data(), fa.trace, sizeof(uint64_t) * ntr, hipMemcpyDeviceToHost));
      (void)hipFree(fa.trace);
      fa.trace = nullptr;
      if (FILE* fp = fopen(ftrace, "wb")) {
        fwrite(hv.data(), sizeof(uint64_t), ntr, fp);
        fclose(fp);
      }
    }
#endif
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    if (early) {   // batch-global stop before imax-1: re-run the batch to L (the kernel exits if L = imax-1)
      fa.unsat = nullptr;
      fa.dL = h->dL;
      HIPCHK(h->timer.timed(0, s, [&] { return launch_fl_fused(fa, h->kind, h->prec, g->dcm, g->dvm, grid, h->f_lds, s); }));
    }
    return IBL_OK;
  }
  if (B <= h->small_b) {
    // small batch: (task, word) items, lane = node (fl_*_small); the per-pass schedule without the fold.
    // Rows packed to the batch (B rounded up to 4 codewords: fl_send's quads, 16-byte pieces) instead of
    // the per-pass path's ldb, so a pass touches E x ldbs elements of each inbox, not one line per edge
    const int nwords = (B + cwl - 1) / cwl, ldbs = (B + 3) / 4 * 4;
    HIPCHK(launch_fl_stage(d_llr, llr_dtype, g->n_v, B, h->chf, h->prec, ldbs, rule, h->bad, s));
    auto grid_of = [&](int ntask) {
      const int need = (ntask * nwords + kFlSmallBlock / 64 - 1) / (kFlSmallBlock / 64);
      return std::max(1, std::min(need, 4 * g->num_cus));
    };
    FlArgs send{};
    send.ch = h->chf; send.out = h->cin; send.start = g->vn_start; send.deg = g->vn_deg; send.tgt = g->tgt_vn;
    send.n_nodes = g->n_v; send.ldb = ldbs; send.B = B;
    FlArgs cn{}, vn{};
    cn.in = h->cin; cn.start = g->cn_start; cn.deg = g->cn_deg; cn.tgt = g->tgt_cn; cn.ch = h->chf;
    vn.out = h->cin; vn.ch = h->chf; vn.start = g->vn_start; vn.deg = g->vn_deg; vn.tgt = g->tgt_vn;
    cn.info = g->cn_info; cn.task = g->cn_task; cn.n_tasks = g->n_cn_task;
    vn.info = g->vn_info; vn.task = g->vn_task; vn.n_tasks = g->n_vn_task;
    cn.llr_max = vn.llr_max = h->llr_max;
    cn.n_nodes = g->n_c; vn.n_nodes = g->n_v;
    cn.nwords = vn.nwords = nwords;
    cn.ldb = vn.ldb = ldbs;
    cn.B = vn.B = B;
    const int gcn = grid_of(g->n_cn_task), gvn = grid_of(g->n_vn_task);
    // the pass chain (decoder buffers only): send, then {CN j, VN j} — replayed from a captured graph (ChainGraphs)
    auto chain = [&](hipStream_t st) -> hipError_t {
      hipError_t e = launch_fl_send(send, h->prec, st);
      if (e != hipSuccess) return e;
      FlArgs c = cn, v = vn;
      for (int j = 1; j < I; ++j) {
        void* vb = (j & 1) ? h->vbuf1 : h->vbuf0;
        c.out = vb;
        c.gate = (early && j >= 3) ? h->flags + (size_t)(j - 2) * kShards : nullptr;
        c.unsat = early ? h->flags + (size_t)(j - 1) * kShards : nullptr;
        if ((e = h->timer.timed(0, st, [&] { return launch_fl_cn_small(c, h->kind, h->prec, g->dcm, gcn, st); })) != hipSuccess)
          return e;
        if (j == I - 1) break;   // the last variable pass feeds no output (as below)
        v.in = vb;
        v.gate = (early && j >= 2) ? h->flags + (size_t)(j - 1) * kShards : nullptr;
        if ((e = h->timer.timed(1, st, [&] { return launch_fl_vn_small(v, h->prec, g->dvm, gvn, st); })) != hipSuccess)
          return e;
      }
      return hipSuccess;
    };
    if (h->s_graphs.on && !h->timer.on) HIPCHK(h->s_graphs.run(B, early ? 1 : 0, s, chain));
    else HIPCHK(chain(s));
    HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
    FlDecArgs dc{};
    dc.vin0 = h->vbuf0; dc.vin1 = h->vbuf1; dc.ch = h->chf; dc.start = g->vn_start; dc.deg = g->vn_deg;
    dc.iters = h->dL; dc.out = d_out; dc.out_dtype = out_dtype; dc.n_nodes = g->n_v; dc.ldb = ldbs; dc.B = B;
    dc.info = g->vn_info; dc.task = g->vn_task; dc.n_tasks = g->n_vn_task; dc.nwords = nwords;
    HIPCHK(launch_fl_dec_small(dc, h->prec, grid_of(g->n_vn_task), s));
    return IBL_OK;
  }
  HIPCHK(launch_fl_stage(d_llr, llr_dtype, g->n_v, B, h->chf, h->prec, h->ldb, rule, h->bad, s));
  FlArgs send{};
  send.ch = h->chf; send.out = h->cin;   // = cb[1] below
  send.start = g->vn_start; send.deg = g->vn_deg; send.tgt = g->tgt_vn;
  send.n_nodes = g->n_v; send.ldb = h->ldb; send.B = B;
  HIPCHK(launch_fl_send(send, h->prec, s));
  // Check pass j reads check inbox cb[j & 1] (send fills cb[1]) and writes the variable inbox vbuf[j & 1];
  // variable pass j writes cb[(j + 1) & 1]. With the fold, check pass j also writes its folded variables'
  // messages into cb[(j + 1) & 1], and the variable pass skips them; the last check pass writes every
  // variable-inbox row (the decision reads them) and folds nothing. The last iteration's variable pass
  // only feeds a syndrome the reference never reads (its loop ends at imax, bp_decoder_irreg.py:240-268),
  // so it is not run.
  if (h->n_folded > 0 && !h->cin2) return fail(IBL_EHIP, "fold inbox missing (fold_alloc)");
  const bool fold = h->n_folded > 0;
  void* cb[2] = {fold ? h->cin2 : h->cin, h->cin};
  FlArgs cn{}, vn{};
  cn.start = g->cn_start; cn.deg = g->cn_deg; cn.tgt = g->tgt_cn; cn.ch = h->chf; cn.fold = h->fold;
  vn.ch = h->chf; vn.start = g->vn_start; vn.deg = g->vn_deg; vn.tgt = g->tgt_vn;
  vn.nodes = fold ? h->vn_nodes : nullptr;
  cn.llr_max = vn.llr_max = h->llr_max;
  cn.n_nodes = g->n_c; vn.n_nodes = fold ? h->n_vn_nodes : g->n_v;
  cn.nchunks = nchunks;
  vn.nchunks = (B + fl_vn_chunk(h->prec, g->dvm) - 1) / fl_vn_chunk(h->prec, g->dvm);
  cn.ldb = vn.ldb = h->ldb;
  cn.B = vn.B = B;
  for (int j = 1; j < I; ++j) {
    void* vb = (j & 1) ? h->vbuf1 : h->vbuf0;
    const bool last = j == I - 1;
    cn.in = cb[j & 1];
    cn.out = vb;
    cn.fout = cb[(j + 1) & 1];
    cn.fold_mode = (fold && !last) ? (early ? 2 : 1) : 0;
    cn.gate = (early && j >= 3) ? h->flags + (size_t)(j - 2) * kShards : nullptr;
    cn.unsat = early ? h->flags + (size_t)(j - 1) * kShards : nullptr;
    HIPCHK(h->timer.timed(0, s, [&] { return launch_fl_cn(cn, h->kind, h->prec, h->g->dcm, h->grid_cn, s); }));
    if (last) break;
    vn.in = vb;
    vn.out = cb[(j + 1) & 1];
    vn.gate = (early && j >= 2) ? h->flags + (size_t)(j - 1) * kShards : nullptr;
    HIPCHK(h->timer.timed(1, s, [&] { return launch_fl_vn(vn, h->prec, h->g->dvm, h->grid_vn, s); }));
  }
  HIPCHK(launch_finalize(h->flags, I, early ? 1 : 0, h->dL, d_iters, s));
  FlDecArgs dc{};
  dc.vin0 = h->vbuf0; dc.vin1 = h->vbuf1; dc.ch = h->chf; dc.start = g->vn_start; dc.deg = g->vn_deg;
  dc.iters = h->dL; dc.out = d_out; dc.out_dtype = out_dtype; dc.n_nodes = g->n_v; dc.nchunks = nchunks;
  dc.ldb = h->ldb; dc.B = B;
  {
    const int n_per = h->prec == kF32 ? 4 : 2;                      // codewords per lane
    const size_t esz = out_dtype == kF32 ? 4 : 8;
    dc.aligned = ((B % n_per) == 0 && ((uintptr_t)d_out % (n_per * esz)) == 0) ? 1 : 0;
    const size_t items = (size_t)g->n_v * nchunks;
    HIPCHK(launch_fl_dec(dc, h->prec, (int)std::min<size_t>((items + 3) / 4, 65536), s));
  }
  return IBL_OK;
}

int ibl_channel_sample(const double* cdf, int32_t T, const double* llr, uint64_t seed, uint64_t offset, int32_t n,
                       int32_t B, const uint8_t* d_bits, void* d_out, int32_t out_dtype, int64_t ld, void* stream) {
  if (!cdf || !d_out) return fail(IBL_EINVAL, "NULL cdf or output");
  if (T < 1 || T > kMaxT) return fail(IBL_EINVAL, "T must lie in [1, 64]");
  if (n < 0 || B < 0) return fail(IBL_EINVAL, "negative shape");
  if (ld < B) return fail(IBL_EINVAL, "ld must be >= B");
  if (out_dtype != kU8 && out_dtype != kI32 && out_dtype != kF32 && out_dtype != kF64)
    return fail(IBL_EINVAL, "unknown output dtype");
  if ((out_dtype == kF32 || out_dtype == kF64) && !llr) return fail(IBL_EINVAL, "LLR output needs llr[T]");
  if (out_dtype == kU8 && T > 256) return fail(IBL_EINVAL, "u8 output needs T <= 256");
  ChArgs a{};
  for (int w = 0; w <= T; ++w) {   // exact: scaling by 2^53 is exact in double; cdf outside [0, 1] saturates
    const double c = std::ldexp(cdf[w], 53);
    a.kthr[w] = std::isnan(c) ? ~0ull : (c <= 0.0 ? 0ull : (c >= 18446744073709551615.0 ? ~0ull : (uint64_t)std::floor(c)));
  }
  if (llr)
    for (int w = 0; w < T; ++w) a.llr[w] = llr[w];
  // binned inversion (sorted thresholds): bin b of m = u 2^53 (b = m >> kChBinSh) holds base = #{w : kthr[w] < bin
  // start} — thresholds every m of the bin exceeds — and n = #{w : kthr[w] inside the bin}, the next n indices
#ifndef IBL_CH_BINNED
#define IBL_CH_BINNED 1   // 0: T compares per sample (A/B, tools/variants.py chloop)
#endif
  a.sorted = IBL_CH_BINNED && std::is_sorted(a.kthr + 1, a.kthr + T + 1) ? 1 : 0;
  if (a.sorted)
    for (int b = 0; b < kChBins; ++b) {
      const uint64_t lo = (uint64_t)b << kChBinSh, hi = lo + (1ull << kChBinSh);
      unsigned base = 0, nin = 0;
      for (int w = 1; w <= T; ++w) {
        base += a.kthr[w] < lo ? 1u : 0u;
        nin += (a.kthr[w] >= lo && a.kthr[w] < hi) ? 1u : 0u;
      }
      a.bin[b] = (uint16_t)(base | (nin << 8));
    }
  a.ctr[0] = offset;
  a.key[0] = seed;
  a.bits = d_bits;
  a.out = d_out;
  a.total = (int64_t)n * B;
  a.ld = ld;
  a.B = B;
  a.T = T;
  a.dtype = out_dtype;
  if (a.total == 0) return IBL_OK;
  HIPCHK(launch_ch_sample(a, (hipStream_t)stream));
  return IBL_OK;
}

// ------------------------------------------------------------------ encoder
}  // extern "C"

struct ibl_encoder {
  int device = 0;
  int32_t N = 0, K = 0, M = 0, max_batch = 0, Bw = 0, method = 0, dir = 1, chain = 0;
  std::string algo;
  int32_t *a_ip = nullptr, *a_ix = nullptr, *l_ip = nullptr, *l_ix = nullptr, *p_ip = nullptr, *p_ix = nullptr;
  int32_t* order = nullptr;
  uint32_t *x = nullptr, *r = nullptr, *t = nullptr, *p = nullptr, *tot = nullptr;
};


extern "C" {

int ibl_encoder_create(int32_t n_v, int32_t n_c, const int32_t* indptr, const int32_t* cols, int32_t max_batch,
                       int32_t device, ibl_encoder** out) {
  if (!out) return fail(IBL_EINVAL, "out is NULL");
  *out = nullptr;
  if (n_v <= n_c || n_c <= 0) return fail(IBL_EINVAL, "H must have fewer rows than columns");
  if (max_batch < 1) return fail(IBL_EINVAL, "max_batch must be >= 1");
  const int32_t N = n_v, M = n_c, K = N - M;
  HIPCHK(hipSetDevice(device));
  EncPlan pl;
  std::string err;
  const int prc = encoder_plan(N, M, indptr, cols, &pl, &err);
  if (prc != 0) return fail(prc == -3 ? IBL_EUNSUPPORTED : IBL_EINVAL, err);
  auto* h = new ibl_encoder();
  h->device = device; h->N = N; h->K = K; h->M = M; h->max_batch = max_batch;
  h->Bw = (max_batch + 31) / 32;
  h->algo = pl.algo;
  h->method = pl.method;
  h->dir = pl.dir;
  h->chain = pl.chain;
  const Csr &A = pl.A, &L = pl.L, &P = pl.P;
  const std::vector<int32_t>& order = pl.order;
  auto bail = [&](int rc) { ibl_encoder_destroy(h); return rc; };
  int rc;
  if ((rc = dupload(&h->a_ip, A.ip.data(), A.ip.size())) || (rc = dupload(&h->a_ix, A.ix.data(), A.ix.size())) ||
      (rc = dupload(&h->p_ip, P.ip.data(), P.ip.size())) || (rc = dupload(&h->p_ix, P.ix.data(), P.ix.size())))
    return bail(rc);
  if (h->method == 1 && ((rc = dupload(&h->l_ip, L.ip.data(), L.ip.size())) || (rc = dupload(&h->l_ix, L.ix.data(), L.ix.size()))))
    return bail(rc);
  if (!order.empty() && (rc = dupload(&h->order, order.data(), order.size()))) return bail(rc);
  const size_t wm = (size_t)M * h->Bw;
  if ((rc = dalloc(&h->x, (size_t)K * h->Bw)) || (rc = dalloc(&h->r, wm)) || (rc = dalloc(&h->t, wm)) ||
      (rc = dalloc(&h->p, wm)) || (rc = dalloc(&h->tot, (size_t)enc_scan_segments() * h->Bw)))
    return bail(rc);
  *out = h;
  return IBL_OK;
}

const char* ibl_encoder_algorithm(const ibl_encoder* h) { return h ? h->algo.c_str() : ""; }

int ibl_encode(ibl_encoder* h, const uint8_t* d_info, int32_t B, uint8_t* d_code, void* stream) {
  if (!h) return fail(IBL_EINVAL, "encoder is NULL");
  if (B < 1 || B > h->max_batch) return fail(IBL_EINVAL, "B must lie in [1, max_batch]");
  if (!d_info || !d_code) return fail(IBL_EINVAL, "NULL buffer");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipSetDevice(h->device));
  const int Bw = (B + 31) / 32, M = h->M;
  HIPCHK(launch_enc_pack(d_info, h->K, B, Bw, h->x, s));
  HIPCHK(launch_enc_ax(h->x, h->a_ip, h->a_ix, M, Bw, h->r, s));
  uint32_t* cur = h->r;
  if (h->method == 1) {                                 // L substitution (forward), then row order
    HIPCHK(launch_enc_subst(cur, h->t, h->l_ip, h->l_ix, M, Bw, 1, s));
    cur = h->t;
  }
  if (h->order) {
    uint32_t* dst = cur == h->r ? h->t : h->r;
    HIPCHK(launch_enc_gather(cur, h->order, M, Bw, dst, s));
    cur = dst;
  }
  if (h->chain) HIPCHK(launch_enc_scan(cur, h->tot, M, Bw, h->dir, h->p, s));
  else HIPCHK(launch_enc_subst(cur, h->p, h->p_ip, h->p_ix, M, Bw, h->dir, s));
  HIPCHK(launch_enc_unpack(d_info, h->p, h->K, M, B, Bw, d_code, s));
  return IBL_OK;
}

void ibl_encoder_destroy(ibl_encoder* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  dfree(h->a_ip); dfree(h->a_ix); dfree(h->l_ip); dfree(h->l_ix); dfree(h->p_ip); dfree(h->p_ix); dfree(h->order);
  dfree(h->x); dfree(h->r); dfree(h->t); dfree(h->p); dfree(h->tot);
  delete h;
}

int ibl_random_bits(uint64_t seed, uint64_t offset, int32_t n, int32_t B, uint8_t* d_out, void* stream) {
  if (!d_out || n < 0 || B < 0) return fail(IBL_EINVAL, "bad arguments");
  if ((int64_t)n * B == 0) return IBL_OK;
  HIPCHK(launch_random_bits(seed, offset, (int64_t)n * B, d_out, (hipStream_t)stream));
  return IBL_OK;
}

int ibl_count_errors(const void* d_x, int32_t dtype, int64_t rows, int32_t B, int64_t ld, double threshold,
                     const uint8_t* d_bits, int64_t bits_ld, int64_t* d_count, void* stream) {
  if (!d_x || !d_bits || !d_count) return fail(IBL_EINVAL, "NULL buffer");
  if (dtype != kU8 && dtype != kI32 && dtype != kF32 && dtype != kF64) return fail(IBL_EINVAL, "unknown dtype");
  if (rows < 0 || B < 0 || ld < B || bits_ld < B) return fail(IBL_EINVAL, "bad shape");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(d_count, 0, sizeof(int64_t), s));
  if (rows * B == 0) return IBL_OK;
  HIPCHK(launch_count_errors(d_x, dtype, rows, B, ld, threshold, d_bits, bits_ld,
                             reinterpret_cast<unsigned long long*>(d_count), s));
  return IBL_OK;
}

int ibl_count_below(const void* d_x, int32_t dtype, int64_t rows, int32_t B, int64_t ld, double threshold,
                    int64_t* d_count, void* stream) {
  if (!d_x || !d_count) return fail(IBL_EINVAL, "NULL buffer");
  if (dtype < kU8 || dtype > kF64) return fail(IBL_EINVAL, "bad dtype");
  if (rows < 0 || B < 0 || ld < B) return fail(IBL_EINVAL, "bad shape");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(d_count, 0, sizeof(int64_t), s));
  if (rows == 0 || B == 0) return IBL_OK;
  HIPCHK(launch_count_below(d_x, dtype, rows, B, ld, threshold, reinterpret_cast<unsigned long long*>(d_count), s));
  return IBL_OK;
}

}  // extern "C"
