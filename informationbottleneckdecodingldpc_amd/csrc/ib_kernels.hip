// Information-bottleneck (integer lookup-table) LDPC decoding kernels for MI355X (gfx950).
//
// Replaces the reference's OpenCL kernels Discrete_LDPC_decoding/kernels_template_irreg.cl
// (and the regular copy kernels_template.cl):
//   checknode_update_iter0 + send_channel_values_to_checknode_inbox  -> ib_cn_fast (pass 0)
//   checknode_update + calc_syndrome + host stop test                -> ib_cn_fast (pass p>=1)
//   varnode_update                                                   -> ib_vn_fast
//   calc_varnode_output                                              -> ib_dec_fast
//
// Fast path design (T_ch == T_dec <= 16, degrees <= kMaxD):
//   * messages are 4-bit nibbles, [edge][codeword] (codeword c in nibble c & 1 of byte c / 2 of its row);
//     a wave item = one node x 1024 codewords (kChunkIB: a lane owns kW = 2 dwords, 16 codewords, of every
//     edge row; the max-degree-16 bodies 1 dword), light variable items (degree <= kLightD) 2048 codewords
//     over 1-KiB row segments (IBL_LIGHT_W); coalesced row segments;
//   * the pass's lookup tables are staged in LDS in quads of 4 (byte slot & 3 of a dword) and super-
//     regions of two quads (common.h quad_off / slot_off), each entry replicated over the 32 banks:
//     entry (t, m) at (t << 12) | (m << 8) | 4 (lane & 31) + slot, so every ds_read_u8 lookup is bank-
//     conflict free and costs one v_lshl_or_b32 (row t merged with the column term) + one DS op, and a
//     column term is one v_perm_b32 placing the codeword's nibble in byte 1 of the lane term (colq);
//   * the order-sensitive folds are computed with prefix sharing (bit-exact: same ops in the
//     same order as the reference's per-output folds, kernels_template_irreg.cl:205-231),
//     25 instead of 35 lookups for a degree-7 check, 35 instead of 56 for a degree-8 variable,
//     list-scheduled onto concurrent chains by tools/gen_sched.py (ib_sched.inc);
//   * the matching step (MATCH, :84-91/:162-172/:233-240) is pre-composed on the host into
//     the final fold table of each degree, so it costs no lookup;
//   * the syndrome of the batch-global early stop (:304-326 + decoder :310-320) is fused
//     into the check-node pass (parity of its inputs), and published as device flags that
//     gate the next launches — no host readback inside the iteration loop.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace ibl {


// LDS lookups take a 32-bit LDS byte address. These kernels have no static LDS, so the dynamic
// array starts at LDS address 0 (checked at kernel entry: lds_at_zero): a lookup is one v_lshl_or
// (row of t merged with the precomputed column term) and one ds_read_u8 whose immediate offset selects
// the table — adding the link-time base of the extern array would cost a second VALU op.
typedef __attribute__((address_space(3))) const uint8_t lds8_t;
// x = row/column part (one v_lshl_or), c = table slot base: x is made opaque so c stays a top-level
// constant and folds into the DS immediate offset instead of being pre-added per input in VGPRs.
__device__ __forceinline__ uint32_t lu(uint32_t x, uint32_t c) {
  asm("" : "+v"(x));
  return *(lds8_t*)(size_t)(x + c);
}
// chained lookup: table value t of the previous step, column term q. The row/column merge is one
// v_lshl_or_b32 per lookup written out, so the compiler cannot hoist t << 12 into a shared
// shift + separate ORs (3 ops for the 2 lookups that read each prefix value P_w).
__device__ __forceinline__ uint32_t luc(uint32_t t, uint32_t q, uint32_t c) {
  uint32_t x;
  static_assert(kRowSh == 12, "luc's shift is the row shift of the table layout");
  asm("v_lshl_or_b32 %0, %1, 12, %2" : "=v"(x) : "v"(t), "v"(q));
  return *(lds8_t*)(size_t)(x + c);
}
// Column fetch (tools/gen_sched.py, "Column fetches"): column T(., m) of one table as 16 nibbles
// (entry t at bits 4t..4t+3), one ds_read_b64 from the bank-replicated column image at byte
// m*256 + 8*(lane&31) of the table's 4-KiB image; cb = 8*(lane&31) + image base. The 32 lanes of a
// bank group read 2 of the 64 banks each: conflict free.
typedef __attribute__((address_space(3))) const uint64_t lds64_t;
__device__ __forceinline__ uint64_t colf(uint32_t m, uint32_t cb) {
  uint32_t x;
  asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(x) : "v"(m), "v"(cb));
  return *(lds64_t*)(size_t)x;
}
// entry t of a fetched column, sh = 4t in its low 6 bits (v_lshrrev_b64 reads only those): a
// previous column result r, whose bits above its nibble hold the next entries, passes as r << 2.
__device__ __forceinline__ uint32_t csel(uint64_t col, uint32_t sh) {
  uint64_t r;
  asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "v"(sh), "v"(col));
  return (uint32_t)r;
}
__device__ __forceinline__ uint32_t lds_base(const uint8_t* p) { return (uint32_t)(size_t)(lds8_t*)p; }
__device__ __forceinline__ void lds_at_zero(const uint8_t* lds) {
  if (lds_base(lds) != 0u) __builtin_trap();  // uniform scalar test; never taken without static LDS
}

// column term of a lookup: (m << 8) | 4*(lane & 31) (+ half / super-region bits); the row term of t is
// t << 12 (common.h, table layout)
__device__ __forceinline__ uint32_t qidx(uint32_t m, uint32_t lane4) { return (m << kColSh) | lane4; }

__device__ __forceinline__ uint32_t valid_mask4(int remaining) {
  return remaining >= 4 ? 0xFu : (remaining <= 0 ? 0u : ((1u << remaining) - 1u));
}

__device__ __forceinline__ bool gate_open(const int32_t* gate, int lane) {
  if (!gate) return true;
  return __ballot(gate[lane] != 0) != 0ull;
}

// img: nreg quads x 256 dwords (dword t*16+m of quad q = entry (t, m) of its 4 tables, common.h layout),
// replicated over the 32 banks. Each wave takes chunks of 64 raw dwords (chunk c -> wave c mod waves); all of
// a lane's raw dwords (up to kStageR chunks) are loaded up front — ONE dependent global round trip — and
// each chunk is written as 8 rounds of ds_write_b128 in which lanes 8i..8i+7 write the 128 bank copies of
// raw dword 8·round + i (fetched with a lane shuffle): consecutive 16-byte units, conflict free. The round-5
// unit loop needed one round trip per 4 units a thread (8 for 3 quads at 256 threads). An odd quad count
// leaves the last super-region's half 1 unwritten (never read).
constexpr int kStageR = 4;
#ifndef IBL_STAGE_UNITS
#define IBL_STAGE_UNITS 0   // 1: the earlier loop, four 16-byte units per thread and round trip (A/B)
#endif
__device__ __forceinline__ void stage_tables(uint8_t* lds, const uint32_t* img, int nreg) {
  if constexpr (IBL_STAGE_UNITS) {
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    const int n = (int)(lds_of_quads(nreg) / 16), bd = blockDim.x;
    for (int u = threadIdx.x; u < n; u += 4 * bd) {
      uint32_t w[4];
      bool ok[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int v = u + k * bd, q = ((v >> 12) << 1) | ((v >> 3) & 1);
        ok[k] = v < n && q < nreg;
        w[k] = ok[k] ? img[q * 256 + ((v >> 4) & 255)] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (ok[k]) l4[u + k * bd] = make_uint4(w[k], w[k], w[k], w[k]);
    }
    return;
  }
  const int nraw = nreg * 256, lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6, nwv = blockDim.x >> 6, nchunk = (nraw + 63) >> 6;
  for (int c0 = 0; c0 < nchunk; c0 += kStageR * nwv) {
    uint32_t v[kStageR];
#pragma unroll
    for (int k = 0; k < kStageR; ++k) {
      const int r = (c0 + wv + k * nwv) * 64 + lane;
      v[k] = r < nraw ? img[r] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kStageR; ++k) {
      const int c = c0 + wv + k * nwv;
      if (c >= nchunk) break;   // wave-uniform
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int src = 8 * p + (lane >> 3), r = c * 64 + src;
        const uint32_t w = __shfl(v[k], src, 64);
        if (r < nraw)
          *reinterpret_cast<uint4*>(lds + quad_off(r >> 8) + (uint32_t)(r & 255) * 256u + 16u * (uint32_t)(lane & 7)) =
              make_uint4(w, w, w, w);
      }
    }
  }
}

// column images: ncs tables x 16 columns x 2 dwords (entries t < 8, t >= 8) replicated for the 32
// lanes of a bank group: LDS dword c*1024 + m*64 + 2*L + h (see colf)
__device__ __forceinline__ void stage_cols(uint8_t* dst, const uint32_t* cimg, int ncs) {
  uint32_t* l32 = reinterpret_cast<uint32_t*>(dst);
  const int n = ncs * 1024;
  for (int i = threadIdx.x; i < n; i += blockDim.x) l32[i] = cimg[((i >> 10) << 5) | (((i >> 6) & 15) << 1) | (i & 1)];
}

// Fast-path message format: T <= 16, so every message is a 4-bit nibble; an edge row stores
// codeword c in nibble (c & 1) of byte c/2. A lane owns 8*W consecutive codewords = W dwords of
// each row (W = rowW<MAXD>()), a wave item = one node x 512*W codewords (256*W-B row segments).
__device__ __forceinline__ uint32_t nib(uint32_t w, int k) { return __builtin_amdgcn_ubfe(w, 4 * k, 4); }
// column term of codeword k of input word w (the generated schedules' form): one v_perm_b32 per codeword
// from the word's even / odd nibbles spread to bytes (w & 0x0F0F0F0F, (w >> 4) & 0x0F0F0F0F, shared by the
// codewords of a group) — bytes 0, 2, 3 from the lane term, byte 1 = the nibble — instead of a v_bfe and a
// v_lshl_or. A/B on one box against the round-4 layout's two ops (profiles/r05_colperm_ab.json):
// C4 176.6k -> 181.0k cw/s, C2 1.791M -> 1.879M. The lane term's byte 1 must be 0 (common.h layout).
__device__ __forceinline__ uint32_t colq(uint32_t w, int k, uint32_t lane4) {
  static_assert(kColSh == 8, "colq places the column in byte 1");
  const uint32_t src = (k & 1) ? ((w >> 4) & 0x0F0F0F0Fu) : (w & 0x0F0F0F0Fu);
  return __builtin_amdgcn_perm(src, lane4, 0x03020000u | ((4u + (uint32_t)(k >> 1)) << 8));
}

// all-ones nibbles for the codewords of a word that lie inside the batch
__device__ __forceinline__ uint32_t valid_nib8(int remaining) {
  return remaining >= 8 ? 0xFFFFFFFFu : (remaining <= 0 ? 0u : ((1u << (4 * remaining)) - 1u));
}

template <int W> struct RowVec;
template <> struct RowVec<1> { typedef uint32_t T; };
template <> struct RowVec<2> { typedef uint2 T; };
template <> struct RowVec<4> { typedef uint4 T; };

// IBL_NT: message rows are streamed once per pass (0.93 GB per inbox at B = 8192, far beyond the
// caches): 1 = nontemporal loads and stores of the variable pass's rows (the HBM-bound pass). The
// check pass keeps plain accesses (its registers are at the cap). A/B on one box (tools/ab.sh, DVB-S2
// B=8192, 2 reps): plain 163.3k cw/s (CN 0.4936 / VN 0.4936 ms), nontemporal 165.3k (0.4888 / 0.4860).
// IBL_NT_CN: the same for the check pass's row loads (not pass 0's channel gather) and stores. Round 4: no
// gain; round 5 on the quad layout (profiles/r05_c4_nontemporal_cn_quad_ab.json): +0.3-0.7 % (the variable
// pass after a nontemporal check pass 0.4257-0.427 vs 0.430 ms), so on by default.
#ifndef IBL_NT_CN
#define IBL_NT_CN 1
#endif
#ifndef IBL_NT
#define IBL_NT 1
#endif
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <int W> struct RowNV;
template <> struct RowNV<1> { typedef uint32_t T; };
template <> struct RowNV<2> { typedef u32x2_t T; };
template <> struct RowNV<4> { typedef u32x4_t T; };

template <int W, bool NT = false>
__device__ __forceinline__ void load_row(const uint8_t* p, uint32_t (&r)[W]) {
  if constexpr (NT) {
    using T = typename RowNV<W>::T;
    const T v = __builtin_nontemporal_load(reinterpret_cast<const T*>(p));
    if constexpr (W == 1) {
      r[0] = v;
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) r[i] = v[i];
    }
  } else {
    const auto v = *reinterpret_cast<const typename RowVec<W>::T*>(p);
    if constexpr (W == 1) {
      r[0] = v;
    } else if constexpr (W == 2) {
      r[0] = v.x; r[1] = v.y;
    } else {
      r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    }
  }
}

template <int W, bool NT = false>
__device__ __forceinline__ void store_row(uint8_t* p, const uint32_t (&r)[W]) {
  if constexpr (NT) {
    using T = typename RowNV<W>::T;
    T v;
    if constexpr (W == 1) {
      v = r[0];
    } else {
#pragma unroll
      for (int i = 0; i < W; ++i) v[i] = r[i];
    }
    __builtin_nontemporal_store(v, reinterpret_cast<T*>(p));
  } else if constexpr (W == 1) {
    *reinterpret_cast<uint32_t*>(p) = r[0];
  } else if constexpr (W == 2) {
    *reinterpret_cast<uint2*>(p) = make_uint2(r[0], r[1]);
  } else {
    *reinterpret_cast<uint4*>(p) = make_uint4(r[0], r[1], r[2], r[3]);
  }
}


// A wave item's inputs, fetched one item ahead of its computation (register double buffer):
// the row loads of item k+1 are issued before item k is computed, so HBM latency overlaps the
// lookups and the waits never cover the previous item's stores.
// Dwords per lane and row: kW for the MAXD=8 bodies; the MAXD=16 bodies already use every VGPR a
// 512-thread block allows and keep one dword (8 codewords) per lane.
template <int MAXD>
constexpr int rowW() { return MAXD <= 8 ? kW : 1; }
template <int MAXD>
constexpr int chunkOf() { return 512 * rowW<MAXD>(); }
static_assert(kLightD <= 8, "light item buffers must fit the MAXD=8 bodies");

template <int MAXD, int W_ = rowW<MAXD>()>
struct ItemBuf {
  static constexpr int kMax = MAXD, W = W_;
  uint32_t row[MAXD][W];   // 8*W packed 4-bit messages (codewords cwb..) of each input row
  uint32_t tgv;            // lane j < d holds the destination row tgt[st + j] of output edge j
  uint32_t chw[W];         // channel values (VN) of the same codewords
  int d, st, node;
  uint32_t off;            // byte offset of this lane's words in a row
  int cwb;                 // first codeword of this lane
};

// Items of a phase: item = first + (pos - pos0) * nch + chunk (nch chunks of 512*W codewords per node)
struct PhaseItems {
  int first, pos0, nch;
};

template <class Buf, bool VN, bool GATHER>
__device__ __forceinline__ void fetch_item(const IbFastArgs& a, int item, int lane, Buf& b, const PhaseItems& pi) {
  constexpr int W = Buf::W, MAXD = Buf::kMax;
  const int rel = item - pi.first;
  const int q = __builtin_amdgcn_readfirstlane(rel / pi.nch);
  const int chunk = __builtin_amdgcn_readfirstlane(rel - q * pi.nch);
  const int pos = pi.pos0 + q;
  const int node = sload(a.info, 4 * pos);
  b.node = node;
  b.st = sload(a.info, 4 * pos + 1);
  b.d = sload(a.info, 4 * pos + 2);
  b.off = (uint32_t)(chunk * (256 * W) + lane * 4 * W);
  b.cwb = chunk * (512 * W) + lane * 8 * W;
  // always MAXD loads (rows past the degree repeat the last row and hit in cache), so the number
  // of outstanding loads is static and the waits stay counted instead of vmcnt(0)
#pragma unroll
  for (int j = 0; j < MAXD; ++j) {
    const int e = b.st + min(j, b.d - 1);
    const uint8_t* row = GATHER ? a.ch8 + (size_t)sload(a.gather, e) * a.ldb : a.in + (size_t)e * a.ldb;
    load_row<W, VN ? (bool)IBL_NT : ((bool)IBL_NT_CN && !GATHER)>(row + b.off, b.row[j]);
  }
  if (VN) {
    load_row<W, IBL_NT>(a.ch8 + (size_t)node * a.ldb + b.off, b.chw);
  } else {
#pragma unroll
    for (int i = 0; i < W; ++i) b.chw[i] = 0;
  }
  // the output-edge targets travel in the same in-order vector-memory stream as the rows, one
  // lane per edge (a scalar load would make the LDS waits conservative); v_readlane at the store
  b.tgv = (uint32_t)a.tgt[b.st + min(lane, b.d - 1)];
}

// Empty asm that consumes every register of a fetched item: the compiler inserts ONE counted
// vmcnt wait for exactly this item's loads here (younger prefetches stay in flight), and no later
// path (switch cases, default) leaves these registers "possibly pending" at a merge point.
template <bool VN, class Buf>
__device__ __forceinline__ void settle(const Buf& b) {
  constexpr int W = Buf::W;
#pragma unroll
  for (int j = 0; j < Buf::kMax; ++j)
#pragma unroll
    for (int i = 0; i < W; ++i) asm volatile("" ::"v"(b.row[j][i]));
  if constexpr (VN) {   // the check pass has no channel words (consuming constant zeros would pin 2W VGPRs)
#pragma unroll
    for (int i = 0; i < W; ++i) asm volatile("" ::"v"(b.chw[i]));
  }
  asm volatile("" ::"v"(b.tgv));
}

// nibbles 4g..4g+3 of an output word
__device__ __forceinline__ uint32_t pack4n(const uint32_t (&t)[4], int g) {
  return (t[0] | (t[1] << 4) | (t[2] << 8) | (t[3] << 12)) << (16 * g);
}

// ------------------------------------------------------------------ check node
// Inputs in_0..in_{D-1} (CN order = ascending column). Output w is the left fold over the
// other inputs with table l at fold step l (kernels_template_irreg.cl:226-231):
//   out[0]   = fold(in_1, in_2, ...),   out[w] = fold(P_w, in_{w+1}, ...),  P_w = fold(in_0..in_{w-1})
// Step l uses LDS slot l, except the last step (l = D-3) which uses fslot (matching composed).
// The chains of one group of cn_sched_s(D) codewords run concurrently per the generated schedule
// (tools/gen_sched.py -> ib_sched.inc: list scheduling of the fold DAG onto L chain lanes).
#ifndef IBL_SCHED_FILE
#define IBL_SCHED_FILE "ib_sched.inc"
#endif
#include IBL_SCHED_FILE

// NCW: codewords of the word that are computed (nibbles 0 .. NCW-1; 4 = the fused kernel's half groups)
template <int D, int NCW = 8>
__device__ __forceinline__ void cn_word(uint32_t lane4, const uint32_t (&in)[D], uint32_t fbase,
                                        const uint32_t (&cb)[4], uint32_t (&outw)[D]) {
#pragma unroll 1   // unrolled (the spread words shared by a word's groups) the check body spills: 56 B at MAXD=8
  for (int k0 = 0; k0 < NCW; k0 += cn_sched_s(D)) cn_group<D>(lane4, in, fbase, cb, outw, k0);
}

// column-image addresses of the column-fetched inputs of a degree-D node (cb of colf)
__device__ __forceinline__ void col_bases(const int8_t (&cc)[4], uint32_t lane8c, uint32_t (&cb)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) cb[i] = lane8c + ((uint32_t)cc[i] << 12);
}

template <int D, bool GATHER, class Buf>
__device__ __forceinline__ void cn_compute(const IbFastArgs& a, uint32_t lane4, uint32_t lane8c, const Buf& b,
                                           int fslot, bool do_par, bool& unsat) {
  constexpr int W = Buf::W;
  uint32_t outw[D][W], trow[D], cb[4];
  col_bases(a.ccol[D], lane8c, cb);
#pragma unroll
  for (int w = 0; w < D; ++w) trow[w] = __builtin_amdgcn_readlane(b.tgv, w);
  const uint32_t fbase = slot_off(fslot);
  if (do_par) {
    // Syndrome of all 8 codewords of a word at once (calc_syndrome, kernels_template_irreg.cl:
    // 304-326: parity of (m < T/2) over the check's inputs). Adding 8 - T/2 to every nibble sets
    // its bit 3 iff m >= T/2 without a carry into the next nibble (m < T <= 16), so the XOR of the
    // D biased words holds in bit 3 of nibble k the parity of (m >= T/2) of codeword k; the parity
    // of (m < T/2) is that XOR (D & 1).
    // The wave's verdict is kept wave-uniform (one ballot per item, SGPRs) rather than as a per-lane
    // flag live across the whole pass.
    const uint32_t bias = (uint32_t)(8 - a.half) * 0x11111111u;
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      uint32_t x = (D & 1) ? 0x88888888u : 0u;
#pragma unroll
      for (int j = 0; j < D; ++j) x ^= b.row[j][i] + bias;
      any |= x & 0x88888888u & valid_nib8(a.B - b.cwb - 8 * i);
    }
    if (__ballot(any != 0) != 0ull) unsat = true;
  }
#pragma unroll
  for (int i = 0; i < W; ++i) {
    uint32_t in[D], o[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      in[j] = b.row[j][i];
      o[j] = 0;
    }
    if constexpr (D == 2) {
      if (a.match) {
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          uint32_t t0[4], t1[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            t0[s] = lu((nib(in[1], 4 * g + s) << kRowSh) + lane4, fbase);
            t1[s] = lu((nib(in[0], 4 * g + s) << kRowSh) + lane4, fbase);
          }
          o[0] |= pack4n(t0, g);
          o[1] |= pack4n(t1, g);
        }
      } else {
        o[0] = in[1];
        o[1] = in[0];
      }
    } else {
      cn_word<D>(lane4, in, fbase, cb, o);
    }
#pragma unroll
    for (int w = 0; w < D; ++w) outw[w][i] = o[w];
  }
#pragma unroll
  for (int w = 0; w < D; ++w) store_row<W, (bool)IBL_NT_CN>(a.out + (size_t)trow[w] * (uint32_t)a.ldb + b.off, outw[w]);
}

// ---------------------------------------------------------------- variable node
// Inputs: channel c and in_0..in_{D-1} (VN order = ascending row). Extrinsic output w folds
// c and the other inputs (kernels_template_irreg.cl:151-160): step 0 = channel table V_0,
// step l = V_l; the last step (l = D-2) uses fslot (matching composed). Degree 1 forwards c
// (:131-136). Schedules as for the check node (vn_group in ib_sched.inc).
template <int D, int NCW = 8>
__device__ __forceinline__ void vn_word(uint32_t lane4, const uint32_t (&in)[D], uint32_t chw,
                                        uint32_t fbase, const uint32_t (&cb)[4], uint32_t (&outw)[D]) {
#pragma unroll 1
  for (int k0 = 0; k0 < NCW; k0 += vn_sched_s(D)) vn_group<D>(lane4, in, chw, fbase, cb, outw, k0);
}

template <int D, class Buf>
__device__ __forceinline__ void vn_compute(const IbFastArgs& a, uint32_t lane4, uint32_t lane8c, const Buf& b,
                                           int fslot) {
  constexpr int W = Buf::W;
  uint32_t outw[D][W], trow[D], cb[4];
  col_bases(a.ccol[D], lane8c, cb);
#pragma unroll
  for (int w = 0; w < D; ++w) trow[w] = __builtin_amdgcn_readlane(b.tgv, w);
  const uint32_t fbase = slot_off(fslot);
#pragma unroll
  for (int i = 0; i < W; ++i) {
    if constexpr (D == 1) {
      outw[0][i] = b.chw[i];
    } else {
      uint32_t in[D], o[D];
#pragma unroll
      for (int j = 0; j < D; ++j) {
        in[j] = b.row[j][i];
        o[j] = 0;
      }
      vn_word<D>(lane4, in, b.chw[i], fbase, cb, o);
#pragma unroll
      for (int w = 0; w < D; ++w) outw[w][i] = o[w];
    }
  }
#pragma unroll
  for (int w = 0; w < D; ++w) store_row<W, IBL_NT>(a.out + (size_t)trow[w] * (uint32_t)a.ldb + b.off, outw[w]);
}

// ------------------------------------------------------------- decision output
// calc_varnode_output (kernels_template_irreg.cl:279-300): fold of channel and ALL inputs with
// the raw tables V_0..V_{D-1} of pass L, no matching. Writes 4 consecutive codewords.
__device__ __forceinline__ void store4(void* out, int dtype, size_t row_off, int cw0, int B, bool aligned,
                                       uint32_t packed) {
  if (dtype == kU8) {
    uint8_t* p = reinterpret_cast<uint8_t*>(out) + row_off + cw0;
    if (aligned && cw0 + 4 <= B) {
      *reinterpret_cast<uint32_t*>(p) = packed;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (cw0 + s < B) p[s] = (uint8_t)(packed >> (8 * s));
    }
  } else {
    int32_t* p = reinterpret_cast<int32_t*>(out) + row_off + cw0;
    if (aligned && cw0 + 4 <= B) {
      int4 v = make_int4(packed & 0xff, (packed >> 8) & 0xff, (packed >> 16) & 0xff, packed >> 24);
      *reinterpret_cast<int4*>(p) = v;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (cw0 + s < B) p[s] = (int32_t)((packed >> (8 * s)) & 0xff);
    }
  }
}

template <int D>
__device__ __forceinline__ void dec_item(const IbDecArgs& a, uint32_t lane4, int node,
                                         int st, uint32_t off, int cwb) {
  uint32_t inw[D];
#pragma unroll
  for (int j = 0; j < D; ++j) inw[j] = *reinterpret_cast<const uint32_t*>(a.vin + (size_t)(st + j) * a.ldb + off);
  const uint32_t cw = *reinterpret_cast<const uint32_t*>(a.ch8 + (size_t)node * a.ldb + off);
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    if (cwb + 4 * g >= a.B) break;   // (wave-uniform in the small-batch kernel: every lane has the same word)
    uint32_t packed = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 4 * g + s;
      uint32_t Q = lu((nib(cw, k) << kRowSh) + qidx(nib(inw[0], k), lane4), 0);
#pragma unroll
      for (int l = 1; l < D; ++l) Q = luc(Q, qidx(nib(inw[l], k), lane4), slot_off(l));
      packed |= Q << (8 * s);
    }
    store4(a.out, a.out_dtype, (size_t)node * a.B, cwb + 4 * g, a.B, a.aligned != 0, packed);
  }
}

// ---------------------------------------------------------------------- kernels
#define IBL_DEG_CASES(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#define IBL_DEG_CASES8(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8)
// Variable-pass co-scheduling (see ib_pass, IBL_MIX16): round-2 A/B on DVB-S2 B=8192 (2 reps each, one box),
// light-first quarters of the block 0: VN 0.4825 ms / 170.4k cw/s, 1: 0.4709 / 171.5k, 2: 0.4703 / 171.8k,
// 3: 0.4782 / 171.1k; round 5 (quad layout): 1 quarter best (IBL_MIX16 = 4).

// LDS of the CN / VN kernels: [nt table quads (common.h layout)][ncs column images][2 work counters]
__device__ __forceinline__ int* lds_counters(const uint8_t* lds, const IbFastArgs& a) {
  return reinterpret_cast<int*>(const_cast<uint8_t*>(lds) + lds_of_quads(a.nt) + (size_t)a.ncs * kColImg);
}
__device__ __forceinline__ void stage_pass(uint8_t* lds, const IbFastArgs& a) {
  if (threadIdx.x < 2) lds_counters(lds, a)[threadIdx.x] = 0;
  stage_tables(lds, a.img, a.nt);
  stage_cols(lds + lds_of_quads(a.nt), a.cimg, a.ncs);
}

// Persistent wave loop shared by the CN and VN passes: items (position, chunk) are dealt
// round-robin to the grid's waves; each iteration prefetches the next item, then computes the
// current one. Degrees dispatch to fully unrolled bodies (wave-uniform switch). Positions are
// heaviest-first: [0, n_heavy) run with a MAXD-row item buffer, the rest with a kLightD-row one
// (a degree-2 node then issues 4 row loads, not MAXD).
// DEPTH: items in flight per wave (2 = ping-pong; 3 for the variable pass's light phase, whose items
// are HBM-bound: A/B on one box, DVB-S2 B=8192, 2 reps: depth 2 VN 0.4618 ms / 174.1k cw/s, depth 3
// 0.4570 ms / 174.7k)
// (with the 1-KiB light rows of IBL_LIGHT_W = 4, depth 2 and 3 measure the same; 2 is the default)
#ifndef IBL_LIGHT_DEPTH
#define IBL_LIGHT_DEPTH 2
#endif
template <class Buf, bool VN, bool GATHER, int DLO, int DEPTH = 2>
__device__ __forceinline__ void ib_phase(const IbFastArgs& a, uint32_t lane4, uint32_t lane8c, int lane, int first,
                                         int end, int nw, int wpb, int* ctr, bool do_par, bool& unsat,
                                         uint64_t* trace_items, const PhaseItems pi) {
  // always inlined: an out-of-line body would take the item by reference through scratch
  auto compute = [&](const Buf& cur) __attribute__((always_inline)) {
    settle<VN>(cur);
    if constexpr (VN) {
      switch (cur.d) {
        case 1: if constexpr (DLO < 1) vn_compute<1>(a, lane4, lane8c, cur, 0); break;
#define X(D) case D: if constexpr (D > DLO && D <= Buf::kMax) vn_compute<D>(a, lane4, lane8c, cur, a.fslot[D]); break;
        IBL_DEG_CASES(X)
#undef X
        default: break;
      }
    } else {
      switch (cur.d) {
#define X(D) case D: if constexpr (D > DLO && D <= Buf::kMax) cn_compute<D, GATHER>(a, lane4, lane8c, cur, a.fslot[D], do_par, unsat); break;
        IBL_DEG_CASES(X)
#undef X
        default: break;
      }
    }
  };
  // Items of this phase: the block owns {first + b*wpb + w + nw*i} (the static round-robin share of
  // its wpb waves), but hands them to its waves dynamically through a workgroup counter in LDS:
  // waves on one SIMD issue oldest-first, so with equal static shares the youngest waves of every
  // CU finished up to 1.5x later than the oldest (traced, IBL_TRACE_WAVES). Ticket k of the block
  // maps to item first + b*wpb + (k % wpb) + nw*(k / wpb). A ticket is taken one item ahead, so
  // the LDS atomic's latency overlaps the current item's lookups.
  // Ping-pong buffers (no register copies: a copy would wait for the prefetched loads); the
  // prefetch is unconditional (clamped to the last item) so the control flow stays straight-line
  // and the compiler's wait for the current item leaves the next item's loads in flight.
  const int base = first + (int)blockIdx.x * wpb;
  auto item_of = [&](int k) { return base + (k % wpb) + nw * (k / wpb); };
  int done = 0;
  if constexpr (DEPTH == 3) {
    // three buffers in rotation (light phase, HBM-bound): item k+2 is fetched before item k is computed
    Buf A, Bb, Cc;
    int ia = item_of(take_ticket(ctr, lane));
    if (ia >= end) return;
    fetch_item<Buf, VN, GATHER>(a, ia, lane, A, pi);
    int ib = item_of(take_ticket(ctr, lane));
    fetch_item<Buf, VN, GATHER>(a, min(ib, end - 1), lane, Bb, pi);
    int kn = take_ticket(ctr, lane);
    for (;;) {
      int ic = item_of(kn);
      fetch_item<Buf, VN, GATHER>(a, min(ic, end - 1), lane, Cc, pi);
      kn = take_ticket(ctr, lane);
      compute(A);
      ++done;
      if (ib >= end) break;
      ia = item_of(kn);
      fetch_item<Buf, VN, GATHER>(a, min(ia, end - 1), lane, A, pi);
      kn = take_ticket(ctr, lane);
      compute(Bb);
      ++done;
      if (ic >= end) break;
      ib = item_of(kn);
      fetch_item<Buf, VN, GATHER>(a, min(ib, end - 1), lane, Bb, pi);
      kn = take_ticket(ctr, lane);
      compute(Cc);
      ++done;
      if (ia >= end) break;
    }
  } else {
    Buf A, Bb;
    int item = item_of(take_ticket(ctr, lane));
    if (item >= end) return;
    fetch_item<Buf, VN, GATHER>(a, item, lane, A, pi);
    int kn = take_ticket(ctr, lane);
    for (;;) {
      int next = item_of(kn);
      fetch_item<Buf, VN, GATHER>(a, min(next, end - 1), lane, Bb, pi);
      kn = take_ticket(ctr, lane);
      compute(A);
      ++done;
      if (next >= end) break;
      item = next;
      next = item_of(kn);
      fetch_item<Buf, VN, GATHER>(a, min(next, end - 1), lane, A, pi);
      kn = take_ticket(ctr, lane);
      compute(Bb);
      ++done;
      if (next >= end) break;
      item = next;
    }
  }
  // trace word {items | cu << 32}: accumulated in memory, not in a register live across the passes
  if (trace_items && lane == 0) *trace_items += (uint64_t)done;
}

// Variable pass, interleaved heavy / light items (IBL_VN_MIX3): every wave runs one heavy item
// (degree > kLightD: LDS-lookup-bound) and two light items (HBM-bound) in turn, so each SIMD always holds both
// kinds. Three buffers in rotation (one heavy, two light — DVB-S2 has 2 light items per heavy one: 51,840 light
// nodes x 4 chunks of 2048 codewords against 12,960 heavy nodes x 8 chunks of 1024): the item computed next is
// always the oldest in flight, so its wait leaves the other two buffers' loads outstanding. When one stream runs
// out the wave computes the buffers it holds and finishes the other stream with the ping-pong phase.
#ifndef IBL_VN_MIX3
#define IBL_VN_MIX3 0
#endif
template <class BufH, class BufL>
__device__ __forceinline__ void ib_phase_mix3(const IbFastArgs& a, uint32_t lane4, uint32_t lane8c, int lane, int hend,
                                              int lend, int nw, int wpb, int* ctr, uint64_t* trace_items,
                                              const PhaseItems pih, const PhaseItems pil) {
  auto compute = [&](const auto& cur) __attribute__((always_inline)) {
    using B = std::decay_t<decltype(cur)>;
    settle<true>(cur);
    switch (cur.d) {
      case 1: if constexpr (B::kMax == kLightD) vn_compute<1>(a, lane4, lane8c, cur, 0); break;
#define X(D) case D: if constexpr (D <= B::kMax && (B::kMax == kLightD || D > kLightD)) vn_compute<D>(a, lane4, lane8c, cur, a.fslot[D]); break;
      IBL_DEG_CASES(X)
#undef X
      default: break;
    }
  };
  const int hbase = (int)blockIdx.x * wpb, lbase = hend + (int)blockIdx.x * wpb;
  auto hitem = [&](int k) { return hbase + (k % wpb) + nw * (k / wpb); };
  auto litem = [&](int k) { return lbase + (k % wpb) + nw * (k / wpb); };
  BufH h;
  BufL l1, l2;
  int ih = hitem(take_ticket(ctr, lane));
  fetch_item<BufH, true, false>(a, min(ih, hend - 1), lane, h, pih);
  int i1 = litem(take_ticket(ctr + 1, lane));
  fetch_item<BufL, true, false>(a, min(i1, lend - 1), lane, l1, pil);
  int i2 = litem(take_ticket(ctr + 1, lane));
  fetch_item<BufL, true, false>(a, min(i2, lend - 1), lane, l2, pil);
  int done = 0;
  for (;;) {
    if (ih >= hend || i1 >= lend || i2 >= lend) break;
    compute(h);
    ih = hitem(take_ticket(ctr, lane));
    fetch_item<BufH, true, false>(a, min(ih, hend - 1), lane, h, pih);
    compute(l1);
    i1 = litem(take_ticket(ctr + 1, lane));
    fetch_item<BufL, true, false>(a, min(i1, lend - 1), lane, l1, pil);
    compute(l2);
    i2 = litem(take_ticket(ctr + 1, lane));
    fetch_item<BufL, true, false>(a, min(i2, lend - 1), lane, l2, pil);
    done += 3;
  }
  // the valid items still held, then whatever is left of either stream
  if (ih < hend) { compute(h); ++done; }
  if (i1 < lend) { compute(l1); ++done; }
  if (i2 < lend) { compute(l2); ++done; }
  if (trace_items && lane == 0) *trace_items += (uint64_t)done;
  bool unsat = false;
  ib_phase<BufH, true, false, kLightD, 2>(a, lane4, lane8c, lane, 0, hend, nw, wpb, ctr, false, unsat, trace_items, pih);
  ib_phase<BufL, true, false, 0, (IBL_LIGHT_DEPTH)>(a, lane4, lane8c, lane, hend, lend, nw, wpb, ctr + 1, false, unsat,
                                                   trace_items, pil);
}

template <int MAXD, bool VN, bool GATHER>
__device__ __forceinline__ void ib_pass(const IbFastArgs& a, const uint8_t* lds) {
  const int lane = threadIdx.x & 63;
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;  // LDS address = byte offset (base checked 0)
  const int wpb = blockDim.x >> 6;
  // wave-uniform item counter: keeps the item loop, the degree switch and the graph-array loads scalar
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6)), nw = gridDim.x * wpb;
  constexpr int W = rowW<MAXD>();
  // the variable pass's light items may use wider rows (IBL_LIGHT_W) and hence fewer chunks per node
  constexpr int LW = (VN && MAXD <= 8) ? IBL_LIGHT_W : W;
  const int nch_l = LW == W ? a.nchunks : (a.B + 512 * LW - 1) / (512 * LW);
  const int heavy_end = a.n_heavy * a.nchunks, nitems = heavy_end + (a.n_nodes - a.n_heavy) * nch_l;
  const bool do_par = !VN && !GATHER && a.unsat != nullptr;   // pass 0 (gather) has no syndrome
  bool unsat = false;
  // trace words written as they arise (start clock, items): values live across the whole pass cost
  // the MAXD=8 check node 2 spilled VGPRs
  uint64_t* trace_items = a.trace ? a.trace + 3 * gw + 2 : nullptr;
  if (a.trace && lane == 0) {
    a.trace[3 * gw] = __builtin_readcyclecounter();
    *trace_items = (uint64_t)__smid() << 32;
  }
  int* ctr = lds_counters(lds, a);  // 2 phase counters
  // column images follow the table quads (colf: cb = 8*(lane&31) + their base + 4 KiB per image)
  const uint32_t lane8c = ((uint32_t)(lane & 31) << 3) + (uint32_t)lds_of_quads(a.nt);
  // Variable passes: heavy items (degree > kLightD) are bound by the LDS array, light ones (DVB-S2's
  // degree-2/3 variables, few lookups per byte moved) by HBM. The first IBL_MIX16 sixteenths of the
  // block's waves take the light share first, so both kinds run side by side on every CU; a wave that
  // exhausts its first share joins the other (two ticket counters). Round 5, quad layout (heavy items
  // now 0.239 ms alone, light 0.2405 ms, together 0.436 ms; profiles/r05_vn_mix_ab.json): a quarter of
  // the waves light-first measured VN 0.4205 ms against 0.433 ms for half (the round-2 choice). Round 6, three
  // alternating repetitions on each of two boxes (profiles/r06_light_first_share_sweep_*.txt): 6 of 16 beat 4 of
  // 16 in all six (C4 +0.26 % / +0.4 %, VN -1 % / -1.5 %); 3, 5, 8 and 10 did not.
#ifndef IBL_MIX16
#define IBL_MIX16 6
#endif
  const bool light_first = VN && (int)(threadIdx.x >> 6) * 16 < wpb * IBL_MIX16;
  if constexpr (VN && MAXD <= 8 && IBL_VN_MIX3) {
    if (a.n_heavy > 0 && a.n_heavy < a.n_nodes) {
      ib_phase_mix3<ItemBuf<MAXD, W>, ItemBuf<kLightD, LW>>(a, lane4, lane8c, lane, heavy_end, nitems, nw, wpb, ctr,
                                                            trace_items, PhaseItems{0, 0, a.nchunks},
                                                            PhaseItems{heavy_end, a.n_heavy, nch_l});
      if (a.trace && lane == 0) a.trace[3 * gw + 1] = __builtin_readcyclecounter();
      return;
    }
  }
#pragma unroll 1
  for (int r = 0; r < 2; ++r) {
    if ((r == 0) != light_first)
      ib_phase<ItemBuf<MAXD, W>, VN, GATHER, kLightD, 2>(a, lane4, lane8c, lane, 0, heavy_end, nw, wpb, ctr, do_par, unsat,
                                                      trace_items, PhaseItems{0, 0, a.nchunks});
    else
      ib_phase<ItemBuf<kLightD, LW>, VN, GATHER, 0, (VN ? IBL_LIGHT_DEPTH : 2)>(a, lane4, lane8c, lane, heavy_end, nitems, nw, wpb, ctr + 1, do_par,
                                                   unsat, trace_items, PhaseItems{heavy_end, a.n_heavy, nch_l});
  }
  if (a.trace && lane == 0) {
    a.trace[3 * gw + 1] = __builtin_readcyclecounter();
  }
  if (do_par && unsat && lane == 0) atomicOr(&a.unsat[gw & (kShards - 1)], 1);
}

// MAXD=16 bodies need more than the 128 VGPRs a 1024-thread block allows: cap those at 512
// threads (256 VGPRs, no scratch spill); the MAXD=8 bodies fit 1024-thread blocks at W <= 2.
// (IBL_LB16 exists for the spill experiment of DESIGN.md "Private segment"; ibl_ib_create refuses
// a build whose fast kernels have a private segment.)
#ifndef IBL_LB8
#define IBL_LB8 1024
#endif
#ifndef IBL_LB16
#define IBL_LB16 512
#endif
// minimum waves per SIMD for the MAXD=8 bodies (register budget 512 / waves); 1 = no constraint
#ifndef IBL_WPE8
#define IBL_WPE8 1
#endif
// check-pass bounds of their own (default: the shared ones): IBL_LB8C / IBL_WPE8C (MAXD=8)
#ifndef IBL_LB8C
#define IBL_LB8C IBL_LB8
#endif
#ifndef IBL_WPE8C
#define IBL_WPE8C IBL_WPE8
#endif
template <int MAXD, bool GATHER>
__global__ __launch_bounds__(MAXD <= 8 ? IBL_LB8C : IBL_LB16, MAXD <= 8 ? IBL_WPE8C : 1) void ib_cn_fast(IbFastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (!gate_open(a.gate, threadIdx.x & 63)) return;  // every wave reads the same words: uniform exit
  lds_at_zero(lds);
  stage_pass(lds, a);
  __syncthreads();
  ib_pass<MAXD, false, GATHER>(a, lds);
}

template <int MAXD>
__global__ __launch_bounds__(MAXD <= 8 ? IBL_LB8 : IBL_LB16, MAXD <= 8 ? IBL_WPE8 : 1) void ib_vn_fast(IbFastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (!gate_open(a.gate, threadIdx.x & 63)) return;
  lds_at_zero(lds);
  stage_pass(lds, a);
  __syncthreads();
  ib_pass<MAXD, true, false>(a, lds);
}

__global__ __launch_bounds__(1024) void ib_dec_fast(IbDecArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const int L = __builtin_amdgcn_readfirstlane(*a.iters);
  lds_at_zero(lds);
  stage_tables(lds, a.img + (size_t)L * a.nt * 256, a.nt);
  __syncthreads();
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;  // LDS address = byte offset (base checked 0)
  const int wpb = blockDim.x >> 6;
  const int gw = blockIdx.x * wpb + (threadIdx.x >> 6), nw = gridDim.x * wpb;
  const int nitems = a.n_nodes * a.nchunks;
  for (int item = gw; item < nitems; item += nw) {
    const int node = __builtin_amdgcn_readfirstlane(item / a.nchunks);
    const int chunk = __builtin_amdgcn_readfirstlane(item - node * a.nchunks);
    const int d = a.deg[node], st = a.start[node];
    const uint32_t off = (uint32_t)(chunk * (kChunkDec / 2) + lane * 4);
    const int cwb = chunk * kChunkDec + lane * 8;
    if (cwb >= a.B) continue;
    switch (d) {
      case 1: dec_item<1>(a, lane4, node, st, off, cwb); break;
#define X(D) case D: dec_item<D>(a, lane4, node, st, off, cwb); break;
      IBL_DEG_CASES(X)
#undef X
      default: break;
    }
  }
}

// ------------------------------------------------------- small-batch per-pass kernels
// The fast kernels' wave item is one node x 512*W codewords: a batch of 2 codewords (the reference's
// DVB-S2 driver, BER_simulation_OpenCL.py:71) leaves all but 2 of those codewords idle, and a pass costs
// what a pass of B = 1024 costs. For batches of a few words a wave item is (task, word) instead: a task is
// up to 64 consecutive positions of one degree in the pass's work order (lane = node, the fused kernel's
// task shape), a word is codewords 8c..8c+7 (one dword of nibbles of every row), each lane gathering its
// node's rows. Same table images, the fused kernel's node bodies on one dword (cn_word / vn_word /
// dec_item), the same syndrome: outputs equal the fast path's bit for bit.
template <int D, bool GATHER>
__device__ __forceinline__ void cn_small_item(const IbFastArgs& a, uint32_t lane4, int st, int c, bool do_par,
                                              bool& unsat) {
  uint32_t in[D], o[D];
  int tg[D];
  const uint32_t off = 4u * (uint32_t)c;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    const int e = st + j;
    const uint8_t* row = GATHER ? a.ch8 + (size_t)a.gather[e] * a.ldb : a.in + (size_t)e * a.ldb;
    in[j] = *reinterpret_cast<const uint32_t*>(row + off);
    tg[j] = a.tgt[e];
    o[j] = 0;
  }
  if (do_par) {   // parity of (m < T/2) over the inputs, 8 codewords at once (see cn_compute)
    const uint32_t bias = (uint32_t)(8 - a.half) * 0x11111111u;
    uint32_t x = (D & 1) ? 0x88888888u : 0u;
#pragma unroll
    for (int j = 0; j < D; ++j) x ^= in[j] + bias;
    if (x & 0x88888888u & valid_nib8(a.B - 8 * c)) unsat = true;
  }
  const uint32_t fbase = slot_off(a.fslot[D]);
  if constexpr (D == 2) {
    if (a.match) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        uint32_t t0[4], t1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          t0[s] = lu((nib(in[1], 4 * g + s) << kRowSh) + lane4, fbase);
          t1[s] = lu((nib(in[0], 4 * g + s) << kRowSh) + lane4, fbase);
        }
        o[0] |= pack4n(t0, g);
        o[1] |= pack4n(t1, g);
      }
    } else {
      o[0] = in[1];
      o[1] = in[0];
    }
  } else {
    const uint32_t cb[4] = {0, 0, 0, 0};   // no column-fetched inputs (the host requires ncs == 0)
    // a word with at most 4 codewords of the batch left (B = 2: every word) computes nibbles 0..3 only
    if (a.B - 8 * c <= 4) cn_word<D, 4>(lane4, in, fbase, cb, o);
    else cn_word<D>(lane4, in, fbase, cb, o);
  }
#pragma unroll
  for (int w = 0; w < D; ++w) *reinterpret_cast<uint32_t*>(a.out + (size_t)tg[w] * a.ldb + off) = o[w];
}

template <int D>
__device__ __forceinline__ void vn_small_item(const IbFastArgs& a, uint32_t lane4, int node, int st, int c) {
  uint32_t in[D], o[D];
  int tg[D];
  const uint32_t off = 4u * (uint32_t)c;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    in[j] = *reinterpret_cast<const uint32_t*>(a.in + (size_t)(st + j) * a.ldb + off);
    tg[j] = a.tgt[st + j];
    o[j] = 0;
  }
  const uint32_t chw = *reinterpret_cast<const uint32_t*>(a.ch8 + (size_t)node * a.ldb + off);
  if constexpr (D == 1) {
    o[0] = chw;   // degree 1 forwards the channel value (kernels_template_irreg.cl:131-136)
  } else {
    const uint32_t cb[4] = {0, 0, 0, 0};
    if (a.B - 8 * c <= 4) vn_word<D, 4>(lane4, in, chw, slot_off(a.fslot[D]), cb, o);
    else vn_word<D>(lane4, in, chw, slot_off(a.fslot[D]), cb, o);
  }
#pragma unroll
  for (int w = 0; w < D; ++w) *reinterpret_cast<uint32_t*>(a.out + (size_t)tg[w] * a.ldb + off) = o[w];
}

// (task, word) items of a small-batch launch, dealt round-robin to the grid's waves; body(node, st, c, d) runs
// for the lanes whose position lies in the task, with this lane's node and first own-order edge. A task
// record {first position, count, degree, contiguous} with contiguous = st0 + 1 says its nodes are
// consecutive with edges st0 + k·d (every DVB-S2 task): the edge then needs no load, and the node (NODE:
// variable passes) one scalar load per task instead of a vector load per lane after the record's.
#ifndef IBL_SMALL_CONTIG
#define IBL_SMALL_CONTIG 1   // 0: every lane loads its node record (A/B, tools/variants.py contig0)
#endif
template <bool NODE, class Args, class Body>
__device__ __forceinline__ void small_items(const Args& a, int lane, Body&& body) {
  const int wpb = blockDim.x >> 6;
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const int nw = gridDim.x * wpb, nitems = a.n_tasks * a.nwords;
  for (int item = gw; item < nitems; item += nw) {
    const int t = __builtin_amdgcn_readfirstlane(item / a.nwords);
    const int c = __builtin_amdgcn_readfirstlane(item - t * a.nwords);
    const int p0 = sload(a.task, 4 * t), cnt = sload(a.task, 4 * t + 1), d = sload(a.task, 4 * t + 2);
    const int st1 = IBL_SMALL_CONTIG ? sload(a.task, 4 * t + 3) : 0;
    if (lane < cnt) {
      int node = 0, st;
      if (st1 != 0) {   // wave-uniform
        st = st1 - 1 + lane * d;
        if constexpr (NODE) node = sload(a.info, 4 * p0) + lane;
      } else {
        st = a.info[4 * (p0 + lane) + 1];
        if constexpr (NODE) node = a.info[4 * (p0 + lane)];
      }
      body(node, st, c, d);
    }
  }
}

template <int MAXD, bool GATHER>
__global__ __launch_bounds__(kSmallBlock) void ib_cn_small(IbFastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  if (!gate_open(a.gate, lane)) return;
  lds_at_zero(lds);
  stage_tables(lds, a.img, a.nt);
  __syncthreads();
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;
  const bool do_par = !GATHER && a.unsat != nullptr;
  bool unsat = false;
  small_items<false>(a, lane, [&](int, int st, int c, int d) __attribute__((always_inline)) {
    switch (d) {
#define X(D) case D: if constexpr (D <= MAXD) cn_small_item<D, GATHER>(a, lane4, st, c, do_par, unsat); break;
      IBL_DEG_CASES(X)
#undef X
      default: break;
    }
  });
  if (do_par && __ballot(unsat) != 0ull && lane == 0)
    atomicOr(&a.unsat[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kShards - 1)], 1);
}

template <int MAXD>
__global__ __launch_bounds__(kSmallBlock) void ib_vn_small(IbFastArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  if (!gate_open(a.gate, lane)) return;
  lds_at_zero(lds);
  stage_tables(lds, a.img, a.nt);
  __syncthreads();
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;
  small_items<true>(a, lane, [&](int node, int st, int c, int d) __attribute__((always_inline)) {
    switch (d) {
      case 1: vn_small_item<1>(a, lane4, node, st, c); break;
#define X(D) case D: if constexpr (D <= MAXD) vn_small_item<D>(a, lane4, node, st, c); break;
      IBL_DEG_CASES(X)
#undef X
      default: break;
    }
  });
}

__global__ __launch_bounds__(kSmallBlock) void ib_dec_small(IbDecArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63;
  const int L = __builtin_amdgcn_readfirstlane(*a.iters);
  lds_at_zero(lds);
  stage_tables(lds, a.img + (size_t)L * a.nt * 256, a.nt);
  __syncthreads();
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;
  small_items<true>(a, lane, [&](int node, int st, int c, int d) __attribute__((always_inline)) {
    const uint32_t off = 4u * (uint32_t)c;
    switch (d) {
      case 1: dec_item<1>(a, lane4, node, st, off, 8 * c); break;
#define X(D) case D: dec_item<D>(a, lane4, node, st, off, 8 * c); break;
      IBL_DEG_CASES(X)
#undef X
      default: break;
    }
  });
}

// ------------------------------------------------------------- fused on-chip decoder
// For short codes (E * 4 B of messages plus the largest pass's table quads within the CU's LDS,
// e.g. regular (3,6) N=8000: 96 KB + 32 KB), one workgroup decodes 8 codewords (a dword of 4-bit
// messages per edge slot) through ALL iterations without touching HBM for messages: the flooding
// schedule of decode_OpenCL (discrete_LDPC_decoder_irreg.py:277-333, kernels_template_irreg.cl)
// as barrier-separated phases over one in-place slot array (a node reads all its inputs before it
// writes its outputs to the same slots):
//   send (:13-31); CN pass 0 (checknode_update_iter0 :33-99); for j = 1..L { VN pass j-1 (:103-179);
//   CN pass j (:181-246) + syndrome of its inputs (:304-326) }; decision with the tables of pass L
//   (calc_varnode_output :249-302).
// The node bodies are the per-pass kernels' (cn_word / vn_word on one dword, the same generated fold
// schedules, the same table images and matching-composed final slots), so outputs equal the per-pass
// path's bit for bit. Tables are staged into the quads at LDS address 0 before every phase (each
// pass has its own tables). Tasks of up to 64 same-degree nodes (lane = node) are handed to waves by
// LDS tickets. Early stop is batch-global: pass 1 runs imax-1 iterations and records each CN pass's
// syndrome in the per-pass path's flag words; finalize_iters turns them into L; pass 2 (dL set)
// re-runs the batch to L only if L < imax-1.
// The fused kernel's light node bodies (checks of degree <= 6, variables <= 4) run every group of the
// dword's 8 codewords unrolled (the per-pass kernels keep `unroll 1` for their register budget; the
// heavier bodies would spill): 2-4x the independent lookup chains per wave,
// which the phase-separated fused schedule needs to keep the LDS busy with 16 waves per CU.
#ifndef IBL_FUSED_UNROLL
#define IBL_FUSED_UNROLL 1
#endif
template <int D, int NCW>
__device__ __forceinline__ void fused_cn_word(uint32_t lane4, const uint32_t (&in)[D], uint32_t fbase,
                                              const uint32_t (&cb)[4], uint32_t (&o)[D]) {
  if constexpr (IBL_FUSED_UNROLL && D <= 6) {
#pragma unroll
    for (int k0 = 0; k0 < NCW; k0 += cn_sched_s(D)) cn_group<D>(lane4, in, fbase, cb, o, k0);
  } else {
    cn_word<D, NCW>(lane4, in, fbase, cb, o);
  }
}
template <int D, int NCW>
__device__ __forceinline__ void fused_vn_word(uint32_t lane4, const uint32_t (&in)[D], uint32_t chw, uint32_t fbase,
                                              const uint32_t (&cb)[4], uint32_t (&o)[D]) {
  if constexpr (IBL_FUSED_UNROLL && D <= 4) {
#pragma unroll
    for (int k0 = 0; k0 < NCW; k0 += vn_sched_s(D)) vn_group<D>(lane4, in, chw, fbase, cb, o, k0);
  } else {
    vn_word<D, NCW>(lane4, in, chw, fbase, cb, o);
  }
}

template <int D, int NCW>
__device__ __forceinline__ void fused_cn_dword(uint32_t* msg, int first, int cnt, int lane, uint32_t lane4,
                                               const IbFusedArgs& a, bool do_par, uint32_t vmask, bool& unsat) {
  uint32_t in[D], o[D];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    in[j] = msg[first + j * cnt + lane];
    o[j] = 0;
  }
  if (do_par) {   // parity of (m < T/2) over the inputs, 8 codewords at once (see cn_compute)
    const uint32_t bias = (uint32_t)(8 - a.half) * 0x11111111u;
    uint32_t x = (D & 1) ? 0x88888888u : 0u;
#pragma unroll
    for (int j = 0; j < D; ++j) x ^= in[j] + bias;
    if (x & 0x88888888u & vmask) unsat = true;
  }
  const uint32_t fbase = slot_off(a.cn_fslot[D]);
  if constexpr (D == 2) {
    if (a.match) {
#pragma unroll
      for (int g = 0; g < NCW / 4; ++g) {
        uint32_t t0[4], t1[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          t0[s] = lu((nib(in[1], 4 * g + s) << kRowSh) + lane4, fbase);
          t1[s] = lu((nib(in[0], 4 * g + s) << kRowSh) + lane4, fbase);
        }
        o[0] |= pack4n(t0, g);
        o[1] |= pack4n(t1, g);
      }
    } else {
      o[0] = in[1];
      o[1] = in[0];
    }
  } else {
    const uint32_t cb[4] = {0, 0, 0, 0};   // no column-fetched inputs (checked on the host: ncs == 0)
    fused_cn_word<D, NCW>(lane4, in, fbase, cb, o);
  }
#pragma unroll
  for (int j = 0; j < D; ++j) msg[first + j * cnt + lane] = o[j];
}

// A variable task's inputs, fetched one task ahead (register double buffer, as ib_phase): slot
// indices of its edges (always MAXD loads, clamped to the degree and to the task's last lane, so
// the number of outstanding loads is static) and the channel dword of its lane's variable.
template <int MAXD>
struct VnTask {
  int pos, cnt, d, sf;
  uint32_t chw;
  int32_t sl[MAXD];
};

template <int MAXD>
__device__ __forceinline__ void fetch_vn_task(const IbFusedArgs& a, const uint32_t* chg, int t, int lane,
                                              VnTask<MAXD>& v, uint32_t csh) {
  if (a.vn_uni) {
    v.pos = 64 * t;
    v.cnt = min(64, a.n_v - v.pos);
    v.d = a.vn_uni;
    v.sf = v.pos * v.d;
  } else {
    v.pos = sload(a.vn_task, 4 * t);
    v.cnt = sload(a.vn_task, 4 * t + 1);
    v.d = sload(a.vn_task, 4 * t + 2);
    v.sf = sload(a.vn_task, 4 * t + 3);
  }
  const int li = min(lane, v.cnt - 1);
  v.chw = chg[v.pos + li] >> csh;   // half groups: this group's 4 codewords into nibbles 0..3
#pragma unroll
  for (int k = 0; k < MAXD; ++k) v.sl[k] = a.vn_slot[v.sf + min(k, v.d - 1) * v.cnt + li];
}

template <int MAXD>
__device__ __forceinline__ void settle_vn(const VnTask<MAXD>& v) {
  asm volatile("" ::"v"(v.chw));
#pragma unroll
  for (int k = 0; k < MAXD; ++k) asm volatile("" ::"v"(v.sl[k]));
}

template <int D, int MAXD, int NCW>
__device__ __forceinline__ void fused_vn_dword(uint32_t* msg, const VnTask<MAXD>& v, uint32_t lane4,
                                               const IbFusedArgs& a) {
  uint32_t in[D], o[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    in[k] = msg[v.sl[k]];
    o[k] = 0;
  }
  if constexpr (D == 1) {
    o[0] = v.chw;     // degree 1 forwards the channel value (:131-136)
  } else {
    const uint32_t cb[4] = {0, 0, 0, 0};
    fused_vn_word<D, NCW>(lane4, in, v.chw, slot_off(a.vn_fslot[D]), cb, o);
  }
#pragma unroll
  for (int k = 0; k < D; ++k) msg[v.sl[k]] = o[k];
}

// decision of one variable for 8 codewords: fold of channel and ALL inputs, raw tables V_0..V_{D-1}
template <int D, int MAXD, int NCW>
__device__ __forceinline__ void fused_dec_dword(const uint32_t* msg, const VnTask<MAXD>& v, uint32_t lane4,
                                                uint32_t (&res)[2]) {
  uint32_t in[D];
#pragma unroll
  for (int k = 0; k < D; ++k) in[k] = msg[v.sl[k]];
#pragma unroll
  for (int g = 0; g < NCW / 4; ++g) {
    uint32_t packed = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 4 * g + s;
      uint32_t Q = lu((nib(v.chw, k) << kRowSh) + qidx(nib(in[0], k), lane4), 0);
#pragma unroll
      for (int l = 1; l < D; ++l) Q = luc(Q, qidx(nib(in[l], k), lane4), slot_off(l));
      packed |= Q << (8 * s);
    }
    res[g] = packed;
  }
}

// Table staging: a pass's raw image is 256 dwords per quad (each entry byte-packed 4 tables deep);
// the LDS image replicates every dword over the 32 banks (common.h layout). Two modes:
// * single set (dbuf = 0): the next phase's raw dwords are loaded into registers at the START of the
//   current phase (2 per thread), written to a small raw buffer in LDS when the wave's tasks are done
//   and replicated LDS -> LDS after the phase barrier (a second barrier follows): the phase boundary
//   pays LDS traffic only, not an L2 round trip;
// * two sets (dbuf = 1, when 2 x nreg quads fit beside the slots, e.g. regular (3,6) N=8000): phase p
//   looks up in set p & 1. A thread loads one source dword per 8 replicated dwords of the next phase's
//   image at the start of the current phase and writes them (two 16-byte stores of the same value) into
//   the other set when its wave's tasks are done, i.e. while slower waves still compute: one barrier per
//   phase and no serial replication step. The set is selected through the lookups' column term (lane4
//   | set offset: bit 7 for one quad a set, bit 16 for two; no extra VALU per lookup).
constexpr int kPfSrc = 2;
struct TablePrefetch {
  uint32_t r[kPfSrc];
  const uint32_t* img;
  int nsrc;   // raw dwords (nt * 256)
  bool dbuf;
  __device__ __forceinline__ void load(const uint32_t* im, int nt) {
    img = im;
    nsrc = nt * 256;
    const int n = dbuf ? nsrc * 4 : nsrc;   // dbuf: units of 8 replicated dwords
#pragma unroll
    for (int k = 0; k < kPfSrc; ++k) {
      const int i = threadIdx.x + k * blockDim.x;
      r[k] = i < n ? img[dbuf ? (i >> 2) : i] : 0u;
    }
  }
  // single set, before the phase barrier: this thread's raw dwords into the raw buffer
  __device__ __forceinline__ void put_raw(uint32_t* raw) const {
#pragma unroll
    for (int k = 0; k < kPfSrc; ++k) {
      const int i = threadIdx.x + k * blockDim.x;
      if (i < nsrc) raw[i] = r[k];
    }
    for (int i = threadIdx.x + kPfSrc * blockDim.x; i < nsrc; i += blockDim.x) raw[i] = img[i];
  }
  // single set, after the phase barrier: replicate the raw buffer (LDS) into the table quads at address 0,
  // one 16-byte unit per thread and round (unit u: super-region u >> 12, row/column (u >> 4) & 255, half
  // (u >> 3) & 1; common.h layout) — LDS reads only, so no prefetched round trips are needed
  __device__ __forceinline__ void replicate(uint8_t* lds, const uint32_t* raw) const {
    const int nreg = nsrc >> 8, n = (int)(lds_of_quads(nreg) / 16);
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    for (int u = threadIdx.x; u < n; u += blockDim.x) {
      const int q = ((u >> 12) << 1) | ((u >> 3) & 1);
      if (q < nreg) {
        const uint32_t w = raw[q * 256 + ((u >> 4) & 255)];
        l4[u] = make_uint4(w, w, w, w);
      }
    }
  }
  // two sets, before the phase barrier: this thread's units straight into the next phase's set, whose
  // quads start at quad fq (unit i = 8 of the 32 bank copies of raw dword i >> 2, common.h layout)
  __device__ __forceinline__ static uint4* unit_at(uint8_t* lds, int fq, int i) {
    const int rr = i >> 2;
    return reinterpret_cast<uint4*>(lds + quad_off(fq + (rr >> 8)) + (uint32_t)(rr & 255) * 256u) + 2 * (i & 3);
  }
  __device__ __forceinline__ void put_set(uint8_t* lds, int fq) const {
    const int n = nsrc * 4;
#pragma unroll
    for (int k = 0; k < kPfSrc; ++k) {
      const int i = threadIdx.x + k * blockDim.x;
      if (i < n) {
        const uint4 v = make_uint4(r[k], r[k], r[k], r[k]);
        uint4* d = unit_at(lds, fq, i);
        d[0] = v;
        d[1] = v;
      }
    }
    for (int i = threadIdx.x + kPfSrc * blockDim.x; i < n; i += blockDim.x) {
      const uint32_t w = img[i >> 2];
      const uint4 v = make_uint4(w, w, w, w);
      uint4* d = unit_at(lds, fq, i);
      d[0] = v;
      d[1] = v;
    }
  }
};

#ifndef IBL_FUSED_TRACE
#define IBL_FUSED_TRACE 0
#endif
// CMAX / VMAX: largest check / variable degree with a body (the variable tasks' index buffers are
// VMAX deep: a (3,6)-regular code runs ib_fused<8, 4>).
// NCW: codewords per workgroup. 8 = a whole dword of nibbles per slot; 4 = half groups for small batches
// (ceil(B/8) below the grid: C1's 1000 codewords fill 125 of 256 CUs at 8): workgroup g decodes
// codewords 4g..4g+3 of the 8-codeword channel group g/2, held in nibbles 0..3 of its slots (the channel
// dword shifted down; nibbles 4..7 stay unused), with half the lookups per node.
template <int CMAX, int VMAX, int NCW = 8>
__global__ __launch_bounds__(CMAX <= 8 && VMAX <= 8 ? 1024 : 512) void ib_fused(IbFusedArgs a) {
  constexpr int MAXD = VMAX;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  lds_at_zero(lds);
  // LDS: [nreg table quads][raw images, nreg x 1 KiB][E message slots][2 counters], or with two
  // table sets (dbuf): [set 0: nreg quads][set 1: nreg quads][E message slots][2 counters]
  // (set 1 = quads nreg..2 nreg-1: at + 128 B for one quad a set, + 64 KiB for two — an offset that adds to
  // every slot's, so it rides in the lanes' column term; the host allows two sets only for nreg <= 2)
  const uint32_t set_off = a.dbuf ? quad_off(a.nreg) : 0u;
  uint32_t* raw = reinterpret_cast<uint32_t*>(lds + lds_of_quads(a.nreg));
  uint32_t* msg = a.dbuf ? reinterpret_cast<uint32_t*>(lds + lds_of_quads(2 * a.nreg)) : raw + (size_t)a.nreg * 256;
  int* ctr = reinterpret_cast<int*>(msg + a.n_e);
  const int lane = threadIdx.x & 63;
  const uint32_t lane4c = (uint32_t)(lane & 31) << 2;
  uint32_t lane4 = lane4c;   // + the set offset of the current phase (dbuf)
  int L = a.imax - 1;
  if (a.dL) {
    L = __builtin_amdgcn_readfirstlane(*a.dL);
    if (L >= a.imax - 1) return;   // no early stop happened: pass 1's outputs stand
  }
  if (threadIdx.x < 2) ctr[threadIdx.x] = 0;
  __syncthreads();
  int ph = 0;
  const int shard = (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kShards - 1));
  TablePrefetch pf;
  pf.dbuf = a.dbuf != 0;
  // end of a phase: the next phase's raw tables into LDS, barrier (every wave done with the old
  // tables and slots), replication, barrier
  // phase trace (diagnostic builds only: -DIBL_FUSED_TRACE=1, tools/variants.py ftrace)
  uint64_t* tr = (IBL_FUSED_TRACE && a.trace && blockIdx.x == 0 && threadIdx.x == 0) ? a.trace : nullptr;
  auto mark = [&](int k) __attribute__((always_inline)) {
    if constexpr (IBL_FUSED_TRACE) {
      if (tr) tr[k] = __builtin_readcyclecounter();
    }
  };
  auto next_phase = [&]() __attribute__((always_inline)) {
    if (pf.dbuf) {
      pf.put_set(lds, ((ph + 1) & 1) ? a.nreg : 0);
      __syncthreads();
      mark(3 * ph + 1);   // all waves done with the phase (and the next phase's set written)
      mark(3 * ph + 2);
    } else {
      pf.put_raw(raw);
      __syncthreads();
      mark(3 * ph + 1);   // all waves done with the phase
      pf.replicate(lds, raw);
      __syncthreads();
      mark(3 * ph + 2);   // next phase's tables staged
    }
    ++ph;
    lane4 = lane4c | ((ph & 1) ? set_off : 0u);
    mark(3 * ph);       // next phase starts
  };
  // check tasks: slots are contiguous per task (no index loads)
  auto cn_phase = [&](bool do_par, uint32_t vmask, bool& unsat) __attribute__((always_inline)) {
    int* c = ctr + (ph & 1);
    if (threadIdx.x == 0) ctr[(ph + 1) & 1] = 0;
    for (;;) {
      const int t = take_ticket(c, lane);
      if (t >= a.n_cn_tasks) break;
      int first, cnt, d;
      if (a.cn_uni) {
        d = a.cn_uni;
        first = 64 * t * d;
        cnt = min(64, a.n_cn_nodes - 64 * t);
      } else {
        first = sload(a.cn_task, 4 * t);
        cnt = sload(a.cn_task, 4 * t + 1);
        d = sload(a.cn_task, 4 * t + 2);
      }
      if (lane < cnt) {
        switch (d) {
#define X(D) case D: if constexpr (D <= CMAX) fused_cn_dword<D, NCW>(msg, first, cnt, lane, lane4, a, do_par, vmask, unsat); break;
          IBL_DEG_CASES(X)
#undef X
          default: break;
        }
      }
    }
  };
  // variable tasks (send / VN pass / decision): task k+1's indices and channel are fetched before task
  // k is computed (ping-pong buffers, unconditional clamped prefetch: straight-line waits)
  auto vn_phase = [&](const uint32_t* chg, uint32_t csh, auto&& body) __attribute__((always_inline)) {
    int* c = ctr + (ph & 1);
    if (threadIdx.x == 0) ctr[(ph + 1) & 1] = 0;
    const int last = a.n_vn_tasks - 1;
    VnTask<MAXD> A, Bb;
    int t = take_ticket(c, lane);
    if (t > last) return;
    fetch_vn_task(a, chg, t, lane, A, csh);
    for (;;) {
      int tn = take_ticket(c, lane);
      fetch_vn_task(a, chg, min(tn, last), lane, Bb, csh);
      settle_vn(A);
      if (lane < A.cnt) body(A);
      if (tn > last) break;
      t = take_ticket(c, lane);
      fetch_vn_task(a, chg, min(t, last), lane, A, csh);
      settle_vn(Bb);
      if (lane < Bb.cnt) body(Bb);
      if (t > last) break;
    }
  };
  constexpr int kSub = 8 / NCW;   // workgroup groups per channel group
  for (int wg = blockIdx.x; wg < a.ngroups * kSub; wg += gridDim.x) {
    const int grp = wg / kSub, sub = wg - grp * kSub;
    const uint32_t* chg = a.chT + (size_t)grp * a.n_v;   // channel by variable position (vn_node order)
    const int cwb = grp * 8 + sub * NCW;
    const uint32_t csh = NCW == 8 ? 0u : (uint32_t)(4 * NCW * sub);
    const uint32_t vmask = valid_nib8(a.B - cwb) & (NCW == 8 ? 0xFFFFFFFFu : 0xFFFFu);
    // send: the channel value to every edge slot of its variable
    mark(0);
    pf.load(a.cn_img, a.cn_nt);
    // (the slot indices are the task's prefetched ones: re-reading them from global memory here put an
    // unprefetched L2 round trip in every task — C1's send phase took 22k cycles against 15k for an
    // iteration's phase)
    vn_phase(chg, csh, [&](const VnTask<MAXD>& v) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < MAXD; ++k)
        if (k < v.d) msg[v.sl[k]] = v.chw;
    });
    next_phase();
    for (int j = 0;; ++j) {
      // CN pass j (tables staged); prefetch the next phase's tables meanwhile
      if (j == L) pf.load(a.dec_img + (size_t)L * a.dec_nt * 256, a.dec_nt);
      else pf.load(a.vn_img + (size_t)j * a.vn_nt * 256, a.vn_nt);
      const bool do_par = j > 0 && a.unsat != nullptr;
      bool unsat = false;
      cn_phase(do_par, vmask, unsat);
      if (do_par && __ballot(unsat) != 0ull && lane == 0) atomicOr(&a.unsat[(size_t)j * kShards + shard], 1);
      next_phase();
      if (j == L) break;
      pf.load(a.cn_img + (size_t)(j + 1) * a.cn_nt * 256, a.cn_nt);
      vn_phase(chg, csh, [&](const VnTask<MAXD>& v) __attribute__((always_inline)) {
        switch (v.d) {
          case 1: fused_vn_dword<1, MAXD, NCW>(msg, v, lane4, a); break;
#define X(D) case D: if constexpr (D <= MAXD) fused_vn_dword<D, MAXD, NCW>(msg, v, lane4, a); break;
          IBL_DEG_CASES(X)
#undef X
          default: break;
        }
      });
      next_phase();
    }
    // decision with the tables of pass L (staged), 8 codewords of one variable per lane
    vn_phase(chg, csh, [&](const VnTask<MAXD>& v) __attribute__((always_inline)) {
      uint32_t r[2] = {0u, 0u};
      switch (v.d) {
        case 1: fused_dec_dword<1, MAXD, NCW>(msg, v, lane4, r); break;
#define X(D) case D: if constexpr (D <= MAXD) fused_dec_dword<D, MAXD, NCW>(msg, v, lane4, r); break;
        IBL_DEG_CASES(X)
#undef X
        default: break;
      }
      const size_t o = (size_t)a.vn_node[v.pos + lane] * a.B + cwb;
      store4(a.out, a.out_dtype, o, 0, a.B - cwb, a.aligned != 0, r[0]);
      if constexpr (NCW == 8) store4(a.out, a.out_dtype, o, 4, a.B - cwb, a.aligned != 0, r[1]);
    });
    __syncthreads();   // every wave done with this group's slots before the next group's send
    mark(3 * ph + 1);
    ++ph;
    lane4 = lane4c | ((ph & 1) ? set_off : 0u);
    tr = nullptr;      // first group only
  }
}

// channel staging for the fused decoder: user [N][B] (u8 / i32) -> chT [group][position] dwords of 8
// nibbles, positions in variable-task order (perm[pos] = node), so a task's lanes read consecutive dwords.
// A cell (position, group) is 8 consecutive codewords of one row: one 8-byte load for aligned u8 rows
// (two 16-byte loads for aligned i32), packed to nibbles in registers (values clamped to 15: cluster ids
// of the fast path's 16-level alphabet); the LDS tile (64 positions x 64 groups, rows padded by one dword)
// only transposes cells, and the dwords are written along the positions.
__global__ __launch_bounds__(256) void ib_stage_t(const void* ch, int dtype, int n, int B, const int32_t* perm,
                                                  uint32_t* chT) {
  constexpr int P = 64, G = 64, RW = G + 1;
  __shared__ uint32_t tile[P * RW];
  const int ngroups = (B + 7) >> 3;
  const int ptiles = (n + P - 1) / P, gtiles = (ngroups + G - 1) / G;
  const uintptr_t base = reinterpret_cast<uintptr_t>(ch);
  const bool vec = (B & 7) == 0 && (dtype == kU8 ? (base & 7) == 0 : (base & 15) == 0);
  auto nib = [](uint32_t x) {   // 4 bytes (each clamped to 15) -> 4 nibbles
    uint32_t y = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) y |= min((x >> (8 * s)) & 0xFFu, 15u) << (4 * s);
    return y;
  };
  for (int t = blockIdx.x; t < ptiles * gtiles; t += gridDim.x) {
    const int p0 = (t % ptiles) * P, g0 = (t / ptiles) * G;
    __syncthreads();
    constexpr int kPer = P * G / 256;   // cells per thread, all loads issued before the LDS stores
    uint32_t w[kPer];
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int i = threadIdx.x + it * 256;
      const int r = i / G, c = i - r * G;
      const int p = p0 + r, g = g0 + c;
      w[it] = 0;
      if (p < n && g < ngroups) {
        const size_t k = (size_t)perm[p] * B + (size_t)g * 8;
        if (vec && dtype == kU8) {
          const uint2 b = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(ch) + k);
          w[it] = nib(b.x) | (nib(b.y) << 16);
        } else if (vec) {
          const int4* q = reinterpret_cast<const int4*>(reinterpret_cast<const int32_t*>(ch) + k);
          const int4 a = q[0], b = q[1];
          const int e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
          for (int s = 0; s < 8; ++s) w[it] |= (uint32_t)min(max(e[s], 0), 15) << (4 * s);
        } else {
#pragma unroll
          for (int s = 0; s < 8; ++s) {
            if (g * 8 + s < B) {
              const int y = dtype == kU8 ? (int)reinterpret_cast<const uint8_t*>(ch)[k + s]
                                         : reinterpret_cast<const int32_t*>(ch)[k + s];
              w[it] |= (uint32_t)min(max(y, 0), 15) << (4 * s);
            }
          }
        }
      }
    }
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int i = threadIdx.x + it * 256;
      const int r = i / G, c = i - r * G;
      tile[r * RW + c] = w[it];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P * G; i += blockDim.x) {
      const int g = i / P, p = i - g * P;
      if (p0 + p < n && g0 + g < ngroups) chT[(size_t)(g0 + g) * n + p0 + p] = tile[p * RW + g];
    }
  }
}

// ------------------------------------------------------ channel staging (u8 / i32 -> u8)
__global__ void ib_stage(const void* ch, int dtype, int n, int B, uint8_t* ch8, int ldb) {
  const int quads = ldb >> 2;
  const size_t total = (size_t)n * quads;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / quads);
    const int cw0 = (int)(i - (size_t)row * quads) * 4;
    uint32_t packed = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int cw = cw0 + s;
      uint32_t v = 0;
      if (cw < B) {
        if (dtype == kU8) {
          v = reinterpret_cast<const uint8_t*>(ch)[(size_t)row * B + cw];
        } else {
          const int32_t x = reinterpret_cast<const int32_t*>(ch)[(size_t)row * B + cw];
          v = (uint32_t)min(max(x, 0), 255);
        }
      }
      packed |= v << (8 * s);
    }
    *reinterpret_cast<uint32_t*>(ch8 + (size_t)row * ldb + cw0) = packed;
  }
}

// ------------------------------------------- channel staging for the fast path (-> 4-bit nibbles)
// Channel staging of the fast path: cluster ids (u8 / i32, [N][B]) -> 4-bit nibbles [N][ldb bytes], the first
// ceil(B / 8) words of every row (the rest of a row is padding no output reads). A block takes one (row, 1024-word
// segment) item at a time: one scalar division per item instead of one 64-bit division per output word (round 6:
// 0.39 -> ~0.1 ms at C4's batch), and rows whose length and base allow it are read as 8 / 32-byte vectors.
__device__ __forceinline__ uint32_t nib8(const uint32_t (&v)[8]) {
  uint32_t p = 0;
#pragma unroll
  for (int s = 0; s < 8; ++s) p |= min(v[s], 15u) << (4 * s);
  return p;
}
template <int DT>
__global__ __launch_bounds__(256) void ib_stage4(const void* ch, int n, int B, uint8_t* ch4, int ldb_bytes, int words,
                                                 int64_t nseg, int vec) {
  constexpr int U = 4;   // words per lane and item
  const int64_t items = (int64_t)n * nseg;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int row = (int)(it / nseg);
    const int seg0 = (int)(it - (int64_t)row * nseg) * (256 * U);
    if constexpr (DT == kU8) {
      // u8 rows of 16-byte multiples (vec == 2) and a whole item inside the row: a lane takes 4 consecutive words
      // (32 codewords) as two 16-byte loads and one 16-byte store (1 KiB per wave instruction)
      if (vec == 2 && seg0 + 256 * U <= words) {
        const int w = seg0 + 4 * (int)threadIdx.x;
        const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(ch) + (size_t)row * B + 8 * (size_t)w);
        const uint4 q0 = p[0], q1 = p[1];
        const uint32_t d[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t e[8];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            e[s] = (d[2 * k] >> (8 * s)) & 0xffu;
            e[4 + s] = (d[2 * k + 1] >> (8 * s)) & 0xffu;
          }
          o[k] = nib8(e);
        }
        *reinterpret_cast<uint4*>(ch4 + (size_t)row * ldb_bytes + 4 * (size_t)w) = make_uint4(o[0], o[1], o[2], o[3]);
        continue;
      }
    }
    const int w0 = seg0 + (int)threadIdx.x;
    uint32_t v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int w = w0 + 256 * u, cw0 = 8 * w;
      if (vec && w < words) {   // B % 8 == 0 and an aligned base: the word's 8 codewords are in the row
        if constexpr (DT == kU8) {
          const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(ch) + (size_t)row * B + cw0);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            v[u][s] = (q.x >> (8 * s)) & 0xffu;
            v[u][4 + s] = (q.y >> (8 * s)) & 0xffu;
          }
        } else {
          const int4* p = reinterpret_cast<const int4*>(reinterpret_cast<const int32_t*>(ch) + (size_t)row * B + cw0);
          const int4 q0 = p[0], q1 = p[1];
          const int32_t x[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
          for (int s = 0; s < 8; ++s) v[u][s] = (uint32_t)min(max(x[s], 0), 255);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int cw = cw0 + s;
          uint32_t e = 0;
          if (w < words && cw < B) {
            if constexpr (DT == kU8) e = reinterpret_cast<const uint8_t*>(ch)[(size_t)row * B + cw];
            else e = (uint32_t)min(max(reinterpret_cast<const int32_t*>(ch)[(size_t)row * B + cw], 0), 255);
          }
          v[u][s] = e;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int w = w0 + 256 * u;
      if (w < words) *reinterpret_cast<uint32_t*>(ch4 + (size_t)row * ldb_bytes + 4 * (size_t)w) = nib8(v[u]);
    }
  }
}

// Small batches (rows of a few words, packed: ldb_bytes = 4 * words): one thread per (row, word), so a block's
// 256 threads write 1 KiB of consecutive staged words instead of one block per row with one busy lane.
template <int DT>
__global__ __launch_bounds__(256) void ib_stage4_words(const void* ch, int n, int B, uint8_t* ch4, int ldb_bytes,
                                                       int words) {
  const int total = n * words;
  for (int i = blockIdx.x * 256 + (int)threadIdx.x; i < total; i += gridDim.x * 256) {
    const int row = i / words, w = i - row * words;
    uint32_t v[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int cw = 8 * w + s;
      uint32_t e = 0;
      if (cw < B) {
        if constexpr (DT == kU8) e = reinterpret_cast<const uint8_t*>(ch)[(size_t)row * B + cw];
        else e = (uint32_t)min(max(reinterpret_cast<const int32_t*>(ch)[(size_t)row * B + cw], 0), 255);
      }
      v[s] = e;
    }
    *reinterpret_cast<uint32_t*>(ch4 + (size_t)row * ldb_bytes + 4 * (size_t)w) = nib8(v);
  }
}

// ----------------------------------------------------------------- generic IB path
// One thread per (node, codeword); reference-exact flat LUT indexing (index clamped to the
// vector so malformed input cannot fault). Used when T_ch != T_dec, T_dec > 16 or a node
// degree exceeds kMaxD.
__device__ __forceinline__ int32_t lut_at(const int32_t* lut, int64_t len, int64_t idx) {
  idx = idx < 0 ? 0 : (idx >= len ? len - 1 : idx);
  return lut[idx];
}

__device__ __forceinline__ uint32_t gen_msg(const IbGenArgs& a, int e, int b) {
  return a.gather ? a.ch8[(size_t)a.gather[e] * a.ldb + b] : a.in[(size_t)e * a.ldb + b];
}

__global__ void ib_cn_gen(IbGenArgs a) {
  const int lane = threadIdx.x & 63;
  if (!gate_open(a.gate, lane)) return;
  const int nb = (a.B + blockDim.x - 1) / blockDim.x;
  bool unsat = false;
  for (int it = blockIdx.x; it < a.n_nodes * nb; it += gridDim.x) {
    const int c = it / nb;
    const int b = (it - c * nb) * blockDim.x + threadIdx.x;
    if (b >= a.B) continue;
    const int d = a.deg[c], st = a.start[c];
    if (a.unsat) {
      uint32_t p = 0;
      for (int w = 0; w < d; ++w) p ^= gen_msg(a, st + w, b) < (uint32_t)a.half;
      unsat |= p != 0;
    }
    const int64_t T = a.T, Tc = a.Tc;
    const int64_t off = Tc * Tc + (int64_t)(a.CM - 3) * Tc * T + (int64_t)(a.pass - 1) * (a.CM - 2) * T * T;
    for (int w = 0; w < d; ++w) {
      auto other = [&](int pos) -> int64_t { return gen_msg(a, st + (pos < w ? pos : pos + 1), b); };
      int64_t x;
      if (a.pass == 0) {
        if (d >= 3) {
          x = lut_at(a.lut, a.lut_len, other(0) * Tc + other(1));
          for (int l = 1; l < d - 2; ++l)
            x = lut_at(a.lut, a.lut_len, x * T + other(l + 1) + Tc * Tc + (int64_t)(l - 1) * Tc * T);
        } else {
          x = other(0);
        }
      } else {
        x = other(0);
        for (int l = 0; l < d - 2; ++l) x = lut_at(a.lut, a.lut_len, off + x * T + other(l + 1) + (int64_t)l * T * T);
      }
      if (a.match) x = lut_at(a.mt, a.mt_len, (int64_t)a.pass * T * a.CM + (int64_t)(d - 1) * T + x);
      a.out[(size_t)a.tgt[st + w] * a.ldb + b] = (uint8_t)x;
    }
  }
  if (a.unsat && __ballot(unsat) != 0ull && lane == 0) atomicOr(&a.unsat[blockIdx.x & (kShards - 1)], 1);
}

__global__ void ib_vn_gen(IbGenArgs a) {
  const int lane = threadIdx.x & 63;
  if (!gate_open(a.gate, lane)) return;
  const int nb = (a.B + blockDim.x - 1) / blockDim.x;
  const int64_t T = a.T, Tc = a.Tc;
  const int64_t off = (int64_t)a.pass * (Tc * T + (int64_t)(a.VM - 1) * T * T);
  for (int it = blockIdx.x; it < a.n_nodes * nb; it += gridDim.x) {
    const int n = it / nb;
    const int b = (it - n * nb) * blockDim.x + threadIdx.x;
    if (b >= a.B) continue;
    const int d = a.deg[n], st = a.start[n];
    const int64_t c = a.ch8[(size_t)n * a.ldb + b];
    if (d == 1) {
      a.out[(size_t)a.tgt[st] * a.ldb + b] = (uint8_t)c;
      continue;
    }
    for (int w = 0; w < d; ++w) {
      auto other = [&](int pos) -> int64_t { return a.in[(size_t)(st + (pos < w ? pos : pos + 1)) * a.ldb + b]; };
      int64_t x = lut_at(a.lut, a.lut_len, off + c * T + other(0));
      for (int l = 1; l <= d - 2; ++l)
        x = lut_at(a.lut, a.lut_len, off + x * T + other(l) + Tc * T + (int64_t)(l - 1) * T * T);
      if (a.match) x = lut_at(a.mt, a.mt_len, (int64_t)a.pass * T * a.VM + (int64_t)(d - 1) * T + x);
      a.out[(size_t)a.tgt[st + w] * a.ldb + b] = (uint8_t)x;
    }
  }
}

__global__ void ib_dec_gen(IbGenDecArgs a) {
  const int nb = (a.B + blockDim.x - 1) / blockDim.x;
  const int L = *a.iters;
  const int64_t T = a.T, Tc = a.Tc;
  const int64_t off = (int64_t)L * (Tc * T + (int64_t)(a.VM - 1) * T * T);
  for (int it = blockIdx.x; it < a.n_nodes * nb; it += gridDim.x) {
    const int n = it / nb;
    const int b = (it - n * nb) * blockDim.x + threadIdx.x;
    if (b >= a.B) continue;
    const int d = a.deg[n], st = a.start[n];
    const int64_t c = a.ch8[(size_t)n * a.ldb + b];
    int64_t x = lut_at(a.lut, a.lut_len, off + c * T + a.vin[(size_t)st * a.ldb + b]);
    for (int l = 1; l < d; ++l)
      x = lut_at(a.lut, a.lut_len, off + x * T + a.vin[(size_t)(st + l) * a.ldb + b] + Tc * T + (int64_t)(l - 1) * T * T);
    if (a.out_dtype == kU8) reinterpret_cast<uint8_t*>(a.out)[(size_t)n * a.B + b] = (uint8_t)x;
    else reinterpret_cast<int32_t*>(a.out)[(size_t)n * a.B + b] = (int32_t)x;
  }
}

// --------------------------------------------------- stop iteration + error counter
// L = first loop iteration j in [1, imax-1] whose flags are all zero (syndrome satisfied),
// else imax-1: the i_num-1 of decode_OpenCL (discrete_LDPC_decoder_irreg.py:277-333).
__global__ void finalize_iters(const int32_t* flags, int imax, int early, int32_t* dL, int32_t* user) {
  const int lane = threadIdx.x & 63;
  int L = imax - 1;
  if (early) {
    for (int j = 1; j <= imax - 1; ++j) {
      if (__ballot(flags[(size_t)j * kShards + lane] != 0) == 0ull) {
        L = j;
        break;
      }
    }
  }
  if (lane == 0) {
    *dL = L;
    if (user) *user = L;
  }
}

// -------------------------------------------------------------------- launchers
hipError_t launch_ib_stage(const void* ch, int dtype, int n, int B, uint8_t* ch8, int ldb, hipStream_t s) {
  const size_t total = (size_t)n * (ldb / 4);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(ib_stage, dim3(grid), dim3(256), 0, s, ch, dtype, n, B, ch8, ldb);
  return hipGetLastError();
}
hipError_t launch_ib_stage4(const void* ch, int dtype, int n, int B, uint8_t* ch4, int ldb_bytes, hipStream_t s) {
  const int words = std::min(ldb_bytes / 4, (B + 7) / 8);
  if (words <= 32 && (int64_t)n * words < (1ll << 31)) {   // small batches: one thread per (row, word)
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(((int64_t)n * words + 255) / 256, 8192));
    if (dtype == kU8)
      hipLaunchKernelGGL(ib_stage4_words<kU8>, dim3(grid), dim3(256), 0, s, ch, n, B, ch4, ldb_bytes, words);
    else
      hipLaunchKernelGGL(ib_stage4_words<kI32>, dim3(grid), dim3(256), 0, s, ch, n, B, ch4, ldb_bytes, words);
    return hipGetLastError();
  }
  const int64_t nseg = (words + 1023) / 1024, items = (int64_t)n * nseg;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(items, 8192));
  const size_t align = dtype == kU8 ? 8 : 16;
  int vec = (B % 8) == 0 && (reinterpret_cast<uintptr_t>(ch) % align) == 0;
  if (vec && dtype == kU8 && (B % 16) == 0 && (reinterpret_cast<uintptr_t>(ch) % 16) == 0 && (ldb_bytes % 16) == 0)
    vec = 2;   // 16-byte rows (ib_stage4's u8 quad-word path)
  if (dtype == kU8)
    hipLaunchKernelGGL(ib_stage4<kU8>, dim3(grid), dim3(256), 0, s, ch, n, B, ch4, ldb_bytes, words, nseg, vec);
  else
    hipLaunchKernelGGL(ib_stage4<kI32>, dim3(grid), dim3(256), 0, s, ch, n, B, ch4, ldb_bytes, words, nseg, vec);
  return hipGetLastError();
}
hipError_t launch_ib_cn_fast(const IbFastArgs& a, int maxd, int grid, int block, size_t lds, hipStream_t s) {
  if (a.gather) {
    if (maxd <= 8) hipLaunchKernelGGL((ib_cn_fast<8, true>), dim3(grid), dim3(block), lds, s, a);
    else hipLaunchKernelGGL((ib_cn_fast<16, true>), dim3(grid), dim3(block), lds, s, a);
  } else {
    if (maxd <= 8) hipLaunchKernelGGL((ib_cn_fast<8, false>), dim3(grid), dim3(block), lds, s, a);
    else hipLaunchKernelGGL((ib_cn_fast<16, false>), dim3(grid), dim3(block), lds, s, a);
  }
  return hipGetLastError();
}
hipError_t launch_ib_vn_fast(const IbFastArgs& a, int maxd, int grid, int block, size_t lds, hipStream_t s) {
  if (maxd <= 8) hipLaunchKernelGGL(ib_vn_fast<8>, dim3(grid), dim3(block), lds, s, a);
  else hipLaunchKernelGGL(ib_vn_fast<16>, dim3(grid), dim3(block), lds, s, a);
  return hipGetLastError();
}
int ib_fast_chunk(int maxd) { return maxd <= 8 ? chunkOf<8>() : chunkOf<16>(); }
static bool ib_small_args_ok(const IbFastArgs& a, bool vn) {
  return a.task && a.info && a.tgt && a.out && a.img && a.ch8 && (a.in || (!vn && a.gather)) && a.n_tasks >= 0 &&
         a.nwords >= 1 && 4 * a.nwords <= a.ldb;
}
hipError_t launch_ib_cn_small(const IbFastArgs& a, int maxd, int grid, size_t lds, hipStream_t s) {
  if (!ib_small_args_ok(a, false)) return hipErrorInvalidValue;
  if (a.gather) {
    if (maxd <= 8) hipLaunchKernelGGL((ib_cn_small<8, true>), dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
    else hipLaunchKernelGGL((ib_cn_small<16, true>), dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
  } else {
    if (maxd <= 8) hipLaunchKernelGGL((ib_cn_small<8, false>), dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
    else hipLaunchKernelGGL((ib_cn_small<16, false>), dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
  }
  return hipGetLastError();
}
hipError_t launch_ib_vn_small(const IbFastArgs& a, int maxd, int grid, size_t lds, hipStream_t s) {
  if (!ib_small_args_ok(a, true)) return hipErrorInvalidValue;
  if (maxd <= 8) hipLaunchKernelGGL(ib_vn_small<8>, dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
  else hipLaunchKernelGGL(ib_vn_small<16>, dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_ib_dec_small(const IbDecArgs& a, int grid, size_t lds, hipStream_t s) {
  if (!a.task || !a.info || !a.vin || !a.img || !a.out || a.nwords < 1 || 4 * a.nwords > a.ldb)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(ib_dec_small, dim3(grid), dim3(small_block(a.nwords)), lds, s, a);
  return hipGetLastError();
}
hipError_t ib_small_private_bytes(int cn_maxd, int vn_maxd, size_t* bytes, const char** name) {
  const bool c8 = cn_maxd <= 8, v8 = vn_maxd <= 8;
  const struct { const void* f; const char* n; } ks[] = {
      {c8 ? (const void*)ib_cn_small<8, true> : (const void*)ib_cn_small<16, true>, "ib_cn_small<gather>"},
      {c8 ? (const void*)ib_cn_small<8, false> : (const void*)ib_cn_small<16, false>, "ib_cn_small"},
      {v8 ? (const void*)ib_vn_small<8> : (const void*)ib_vn_small<16>, "ib_vn_small"},
      {(const void*)ib_dec_small, "ib_dec_small"}};
  *bytes = 0;
  *name = "";
  for (const auto& k : ks) {
    hipError_t e = hipFuncSetAttribute(k.f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e != hipSuccess) return e;
    hipFuncAttributes fa;
    e = hipFuncGetAttributes(&fa, k.f);
    if (e != hipSuccess) return e;
    if (fa.localSizeBytes > *bytes) {
      *bytes = fa.localSizeBytes;
      *name = k.n;
    }
  }
  return hipSuccess;
}
hipError_t launch_ib_dec_fast(const IbDecArgs& a, int grid, int block, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(ib_dec_fast, dim3(grid), dim3(block), lds, s, a);
  return hipGetLastError();
}
hipError_t ib_fast_occupancy(int which, int maxd, int block, size_t lds, int* blocks_per_cu) {
  if (which == 0) {  // every variant must accept the LDS size; report the non-gather one
    for (const void* g : {(const void*)ib_cn_fast<8, true>, (const void*)ib_cn_fast<16, true>}) {
      hipError_t e = hipFuncSetAttribute(g, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
      if (e != hipSuccess) return e;
    }
  }
  const void* f = which == 0 ? (maxd <= 8 ? (const void*)ib_cn_fast<8, false> : (const void*)ib_cn_fast<16, false>)
                : which == 1 ? (maxd <= 8 ? (const void*)ib_vn_fast<8> : (const void*)ib_vn_fast<16>)
                             : (const void*)ib_dec_fast;
  hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (e != hipSuccess) return e;
  hipFuncAttributes fa;
  e = hipFuncGetAttributes(&fa, f);
  if (e != hipSuccess) return e;
  if (block > fa.maxThreadsPerBlock) return hipErrorInvalidValue;  // above the kernel's launch bounds
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, block, lds);
}
hipError_t ib_fast_private_bytes(int cn_maxd, int vn_maxd, size_t* bytes, const char** name) {
  const bool c8 = cn_maxd <= 8, v8 = vn_maxd <= 8;
  const struct { const void* f; const char* n; } ks[] = {
      {c8 ? (const void*)ib_cn_fast<8, true> : (const void*)ib_cn_fast<16, true>, c8 ? "ib_cn_fast<8,gather>" : "ib_cn_fast<16,gather>"},
      {c8 ? (const void*)ib_cn_fast<8, false> : (const void*)ib_cn_fast<16, false>, c8 ? "ib_cn_fast<8>" : "ib_cn_fast<16>"},
      {v8 ? (const void*)ib_vn_fast<8> : (const void*)ib_vn_fast<16>, v8 ? "ib_vn_fast<8>" : "ib_vn_fast<16>"},
      {(const void*)ib_dec_fast, "ib_dec_fast"}};
  *bytes = 0;
  *name = "";
  for (const auto& k : ks) {
    hipFuncAttributes fa;
    const hipError_t e = hipFuncGetAttributes(&fa, k.f);
    if (e != hipSuccess) return e;
    if (fa.localSizeBytes > *bytes) {
      *bytes = fa.localSizeBytes;
      *name = k.n;
    }
  }
  return hipSuccess;
}
hipError_t launch_ib_stage_t(const void* ch, int dtype, int n, int B, const int32_t* perm, uint32_t* chT,
                             hipStream_t s) {
  const size_t tiles = (size_t)((n + 63) / 64) * (size_t)((((B + 7) >> 3) + 63) / 64);
  const int grid = (int)std::max<size_t>(1, std::min<size_t>(tiles, 8192));
  hipLaunchKernelGGL(ib_stage_t, dim3(grid), dim3(256), 0, s, ch, dtype, n, B, perm, chT);
  return hipGetLastError();
}
static const void* ib_fused_kernel(int cmax, int vmax, int ncw) {
  if (ncw == 4) {
    if (cmax <= 8 && vmax <= 4) return (const void*)ib_fused<8, 4, 4>;
    if (cmax <= 8 && vmax <= 8) return (const void*)ib_fused<8, 8, 4>;
    return (const void*)ib_fused<16, 16, 4>;
  }
  if (cmax <= 8 && vmax <= 4) return (const void*)ib_fused<8, 4>;
  if (cmax <= 8 && vmax <= 8) return (const void*)ib_fused<8, 8>;
  return (const void*)ib_fused<16, 16>;
}
hipError_t launch_ib_fused(const IbFusedArgs& a, int cmax, int vmax, int grid, int block, size_t lds, hipStream_t s) {
  IbFusedArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(ib_fused_kernel(cmax, vmax, a.ncw), dim3(grid), dim3(block), p, lds, s);
}
hipError_t ib_fused_occupancy(int cmax, int vmax, int ncw, size_t lds, int* blocks_per_cu, int* block,
                              size_t* private_bytes) {
  const void* f = ib_fused_kernel(cmax, vmax, ncw);
  // the dynamic-LDS cap is an attribute of the kernel instantiation, shared by every decoder that launches it:
  // set it to the CU's whole LDS (here and in the other *_occupancy functions), never to one decoder's size,
  // or a smaller decoder created later would lower the cap an earlier, larger one launches with
  hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (e != hipSuccess) return e;
  hipFuncAttributes fa;
  if ((e = hipFuncGetAttributes(&fa, f)) != hipSuccess) return e;
  *block = cmax <= 8 && vmax <= 8 ? 1024 : 512;
  *private_bytes = fa.localSizeBytes;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, *block, lds);
}
static int gen_grid(int n_nodes, int B) {
  const long long items = (long long)n_nodes * ((B + 255) / 256);
  return (int)std::min<long long>(items, 65536);
}
hipError_t launch_ib_cn_gen(const IbGenArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ib_cn_gen, dim3(gen_grid(a.n_nodes, a.B)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_ib_vn_gen(const IbGenArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ib_vn_gen, dim3(gen_grid(a.n_nodes, a.B)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_ib_dec_gen(const IbGenDecArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ib_dec_gen, dim3(gen_grid(a.n_nodes, a.B)), dim3(256), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_finalize(const int32_t* flags, int imax, int early, int32_t* dL, int32_t* user, hipStream_t s) {
  hipLaunchKernelGGL(finalize_iters, dim3(1), dim3(64), 0, s, flags, imax, early, dL, user);
  return hipGetLastError();
}

}  // namespace ibl
