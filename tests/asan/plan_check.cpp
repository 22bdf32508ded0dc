// CPU-only checker of the C ABI's host planning code (informationbottleneckdecodingldpc_amd/csrc/plan.h),
// built by tests/test_cpu_host.py with -fsanitize=address,undefined -fno-sanitize-recover=all, so any
// out-of-bounds access, use-after-free, leak or undefined behaviour in the planning code fails the test.
//
//   plan_check <graph.bin>
// graph.bin: int32 n_v, n_c, indptr[n_c + 1], cols[E] (canonical CSR of H). Runs every planning step the
// decoders and the encoder take at create time — map_node_connections, the fast path's work orders and
// small-batch tasks, the float fold plan, the fused kernels' task tables (both variable orders, two scan
// windows) with the float kernel's padding, the encoder plan — checks their invariants and prints one JSON
// line of what they derived. Exit status 0 = every invariant held.
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

#include "plan.h"

using namespace ibl;

static int g_fail = 0;
#define CHECK(cond, what)                                              \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "invariant failed: %s (%s)\n", what, #cond); \
      ++g_fail;                                                        \
    }                                                                  \
  } while (0)

static bool is_perm(const std::vector<int32_t>& v, size_t n) {
  if (v.size() != n) return false;
  std::vector<char> seen(n, 0);
  for (int32_t x : v) {
    if (x < 0 || (size_t)x >= n || seen[x]) return false;
    seen[x] = 1;
  }
  return true;
}

// work order + tasks of one side: a permutation of the nodes, heaviest first; tasks cover it in order
static void check_side(const std::vector<int32_t>& start, const std::vector<int32_t>& deg, const char* side) {
  int32_t heavy = -1;
  const std::vector<int32_t> info = work_order(start, deg, &heavy);
  const size_t n = deg.size();
  std::vector<int32_t> nodes(n);
  int32_t h = 0;
  for (size_t p = 0; p < n; ++p) {
    nodes[p] = info[4 * p];
    CHECK(info[4 * p + 1] == start[info[4 * p]] && info[4 * p + 2] == deg[info[4 * p]], side);
    if (p) CHECK(info[4 * p + 2] <= info[4 * (p - 1) + 2], side);
    h += deg[info[4 * p]] > kLightD;
  }
  CHECK(is_perm(nodes, n), side);
  CHECK(h == heavy, side);
  const std::vector<int32_t> t = order_tasks(info);
  size_t pos = 0;
  for (size_t k = 0; k < t.size() / 4; ++k) {
    const int32_t p0 = t[4 * k], c = t[4 * k + 1], d = t[4 * k + 2], ct = t[4 * k + 3];
    CHECK(p0 == (int32_t)pos && c >= 1 && c <= 64, side);
    for (int32_t i = 0; i < c; ++i) CHECK(info[4 * (p0 + i) + 2] == d, side);
    if (ct) {
      for (int32_t i = 0; i < c; ++i)
        CHECK(info[4 * (p0 + i)] == info[4 * p0] + i && info[4 * (p0 + i) + 1] == ct - 1 + i * d, side);
    }
    pos += c;
  }
  CHECK(pos == n, side);
}

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: plan_check graph.bin\n");
    return 2;
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hdr[2];
  if (std::fread(hdr, 4, 2, f) != 2) return 2;
  const int32_t n_v = hdr[0], n_c = hdr[1];
  std::vector<int32_t> indptr(n_c + 1);
  if (std::fread(indptr.data(), 4, indptr.size(), f) != indptr.size()) return 2;
  std::vector<int32_t> cols(indptr[n_c]);
  if (std::fread(cols.data(), 4, cols.size(), f) != cols.size()) return 2;
  std::fclose(f);
  const int64_t E = indptr[n_c];

  HostGraph g;
  g.n_v = n_v;
  g.n_c = n_c;
  g.n_e = E;
  g.h_cn_start.resize(n_c);
  g.h_cn_deg.resize(n_c);
  g.h_vn_start.resize(n_v);
  g.h_vn_deg.resize(n_v);
  g.h_tgt_vn.resize(E);
  std::vector<int32_t> tgt_cn(E);
  std::string err;
  if (!map_node_connections(n_v, n_c, indptr.data(), cols.data(), g.h_cn_start.data(), g.h_cn_deg.data(),
                            tgt_cn.data(), g.h_vn_start.data(), g.h_vn_deg.data(), g.h_tgt_vn.data(), &err)) {
    std::fprintf(stderr, "map_node_connections: %s\n", err.c_str());
    return 1;
  }
  g.h_cols = cols;
  for (int64_t e = 0; e < E; ++e) CHECK(g.h_tgt_vn[tgt_cn[e]] == e, "tgt_vn o tgt_cn = id");
  CHECK(std::accumulate(g.h_vn_deg.begin(), g.h_vn_deg.end(), (int64_t)0) == E, "variable degrees sum to E");
  {   // a malformed CSR is refused, not read out of bounds
    std::vector<int32_t> bad(cols);
    if (!bad.empty()) bad[0] = n_v;
    std::vector<int32_t> a(n_c), b(n_c), c(E), d(n_v), e(n_v), t(E);
    CHECK(!map_node_connections(n_v, n_c, indptr.data(), bad.data(), a.data(), b.data(), c.data(), d.data(),
                                e.data(), t.data(), &err), "out-of-range column refused");
  }
  check_side(g.h_cn_start, g.h_cn_deg, "check side");
  check_side(g.h_vn_start, g.h_vn_deg, "variable side");

  // float fold plan: every folded variable sits in two check records, the rest is the complement
  std::vector<int32_t> rec, rest;
  const int32_t nf = plan_fold(g, &rec, &rest);
  {
    std::vector<int32_t> cnt(n_v, 0);
    for (int32_t c = 0; c < n_c; ++c)
      for (int k = 0; k < 2; ++k) {
        const int32_t p = rec[(size_t)kFoldRec * c + k];
        if (p < 0) continue;
        CHECK(p < g.h_cn_deg[c], "fold position inside its check");
        const int32_t v = rec[(size_t)kFoldRec * c + 4 + k];
        CHECK(v >= 0 && v < n_v && g.h_vn_deg[v] == 2, "folded variable has degree 2");
        CHECK(cols[g.h_cn_start[c] + p] == v, "fold record names the variable at its position");
        const int32_t other = rec[(size_t)kFoldRec * c + 2 + k];
        CHECK(other >= 0 && other < E && cols[other] == v && other != g.h_cn_start[c] + p, "other edge of v");
        ++cnt[v];
      }
    int32_t folded = 0;
    for (int32_t v = 0; v < n_v; ++v) {
      CHECK(cnt[v] == 0 || cnt[v] == 2, "a folded variable has two records");
      folded += cnt[v] == 2;
    }
    CHECK(folded == nf && (int32_t)rest.size() == n_v - nf, "fold count");
  }

  // fused task tables: check slots form a permutation of [0, E); every variable edge maps to its own slot
  int32_t ncn_task = 0, nvn_task = 0;
  size_t padded = 0;
  for (int mode = 0; mode < 3; ++mode) {
    FusedTasks ft;
    build_fused_tasks(g, &ft, mode > 0, mode == 2 ? (size_t)1 << 30 : 256);
    std::vector<int32_t> slot_of_edge(E, -1);
    int64_t covered = 0;
    for (size_t t = 0; t < ft.cn_task.size() / 4; ++t) covered += (int64_t)ft.cn_task[4 * t + 1] * ft.cn_task[4 * t + 2];
    CHECK(covered == E, "check tasks cover every edge");
    CHECK(is_perm(ft.vn_node, n_v), "variable task order is a permutation");
    std::vector<int32_t> slots(ft.vn_slot);
    CHECK(is_perm(slots, (size_t)E), "variable-edge slots are a permutation of the check slots");
    for (size_t t = 0; t < ft.vn_task.size() / 4; ++t) {
      const int32_t p0 = ft.vn_task[4 * t], c = ft.vn_task[4 * t + 1], d = ft.vn_task[4 * t + 2];
      for (int32_t i = 0; i < c; ++i) CHECK(g.h_vn_deg[ft.vn_node[p0 + i]] == d, "variable task degree");
    }
    ncn_task = (int32_t)(ft.cn_task.size() / 4);
    nvn_task = (int32_t)(ft.vn_task.size() / 4);
    pad_vn_slots(&ft);
    size_t want = 0;
    for (size_t t = 0; t < ft.vn_task.size() / 4; ++t) want += (size_t)64 * ft.vn_task[4 * t + 2];
    CHECK(ft.vn_slot.size() == want, "padded slot rows");
    padded = want;
  }

  // encoder plan (H = [A | B]; refused when B is singular)
  EncPlan pl;
  const int erc = n_v > n_c ? encoder_plan(n_v, n_c, indptr.data(), cols.data(), &pl, &err) : -1;
  if (erc == 0) {
    CHECK((int32_t)pl.A.ip.size() == n_c + 1 && (int32_t)pl.P.ip.size() == n_c + 1, "plan rows");
    for (int32_t x : pl.P.ix) CHECK(x >= 0 && x < n_c, "P columns");
    if (!pl.order.empty()) CHECK(is_perm(pl.order, (size_t)n_c), "row order is a permutation");
  }
  std::printf("{\"n_v\": %d, \"n_c\": %d, \"n_e\": %lld, \"folded\": %d, \"cn_tasks\": %d, \"vn_tasks\": %d, "
              "\"padded_slots\": %zu, \"encoder_rc\": %d, \"algo\": \"%s\", \"chain\": %d, \"failures\": %d}\n",
              n_v, n_c, (long long)E, nf, ncn_task, nvn_task, padded, erc, erc == 0 ? pl.algo.c_str() : "",
              erc == 0 ? pl.chain : 0, g_fail);
  return g_fail ? 1 : 0;
}
