// Shared definitions for the MI355X (gfx950) LDPC decoding kernels.
//
// Message layout: every inbox is [edge][codeword] with a padded row stride `ldb`
// (codeword-minor, like the reference's inbox buffers, discrete_LDPC_decoder_irreg.py:214-219),
// so the lanes of a wavefront touch consecutive codewords of one edge row: one 256-B (u8) or
// 1-KiB (fp32) coalesced segment per row and wave.  A "wave item" is one node × one chunk of
// kChunk codewords.
#pragma once
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <stddef.h>
#include <stdint.h>

#include "plan.h"

namespace ibl {

constexpr int kWave = 64;
constexpr int kChunk = 256;       // codewords per wave item (fp32: 4 per lane, fp64: 2x2)
// IB fast path: 4-bit messages; a lane owns IBL_W dwords (8*IBL_W codewords) of each edge row
#ifndef IBL_W
#define IBL_W 2
#endif
constexpr int kW = IBL_W;
constexpr int kChunkIB = 512 * kW;  // codewords per fast-path wave item
// IBL_LIGHT_W: dwords per lane and row of the variable pass's light items (degree <= kLightD; the
// MAXD=8 bodies): 4 = 1-KiB row segments per wave, chunks of 2048 codewords. A/B on one box (DVB-S2
// B=8192, 2 reps, tools/r03f.sh): light W=2 with 3 items in flight VN 0.4737 ms / 168.6k cw/s, W=4
// with 3 in flight 0.4594 / 170.7k, W=4 with 2 in flight 0.4583 / 170.9k (the default)
#ifndef IBL_LIGHT_W
#define IBL_LIGHT_W 4
#endif
constexpr int kRowPad = 512 * (IBL_LIGHT_W > IBL_W ? IBL_LIGHT_W : IBL_W);   // row padding (codewords)
constexpr int kChunkDec = 512;      // codewords per decision-kernel wave item
constexpr int kTbl = 8192;        // LDS bytes per IB lookup table (replicated over the 32 banks)
// LDS table layout (round 5): tables in quads of 4 — byte (slot & 3) of a dword holds table `slot` —
// and two quads per 64-KiB super-region, interleaved at 128 B: quad q lives in super-region q >> 1,
// half q & 1 (address bit 7). Entry (t, m) of a table sits at row t (4 KiB stride), column m (256 B),
// replicated for the 32 banks (lane & 31), so a lookup address is
//   (t << 12) | (m << 8) | 4*(lane&31) + slot_off(slot)
// with the slot in the DS immediate for slots < 8. Byte 1 of an address is the column alone, so a
// column term is one v_perm_b32 that drops a codeword's nibble (spread to a byte) into byte 1 of the
// lane term (colq); bytes 0, 2, 3 keep the lane, half and super-region bits.
constexpr int kSuper = 65536;                 // bytes per super-region (2 quads)
constexpr int kRowSh = 12, kColSh = 8;        // row / column shifts of a lookup address
__host__ __device__ constexpr uint32_t quad_off(int q) { return (uint32_t)(q >> 1) * kSuper + (uint32_t)(q & 1) * 128u; }
__host__ __device__ constexpr uint32_t slot_off(int s) { return quad_off(s >> 2) + (uint32_t)(s & 3); }
constexpr int regions_of(int nt) { return (nt + 3) >> 2; }   // quads of nt tables
// LDS bytes of nq quads from address 0 (an odd count leaves the last super-region's half 1 unused)
__host__ __device__ constexpr size_t lds_of_quads(int nq) { return (size_t)((nq + 1) >> 1) * kSuper; }
// Column images (tools/gen_sched.py "Column fetches"): the last cn_ncols(D) / vn_ncols(D) inputs of a
// node read their shared table's whole column (16 nibbles, ds_read_b64) instead of one entry per
// chain. 4 KiB of LDS per table image (16 columns x 32 lane copies x 8 B).
constexpr int kColImg = 4096;
#ifndef IBL_NC_CN
#define IBL_NC_CN 0
#endif
#ifndef IBL_NC_VN
#define IBL_NC_VN 0
#endif
__host__ __device__ constexpr int cn_ncols(int D) { return (D >= 5 && D <= 8) ? IBL_NC_CN : 0; }
__host__ __device__ constexpr int vn_ncols(int D) { return (D >= 6 && D <= 8) ? IBL_NC_VN : 0; }
constexpr int kTP = 16;           // IB fast path: alphabet padded to 16 (entry (t,m) at t*16+m)
// kMaxD, kLightD, kFoldRec: plan.h
constexpr int kShards = 64;       // early-stop flag words per iteration (one wave load)
constexpr int kLdsBytes = 160 * 1024;

enum Dtype : int32_t { kU8 = 1, kI32 = 2, kF32 = 3, kF64 = 4 };

// the C ABI's per-thread last error (capi.hip; ibl_last_error): other translation units report through it
int set_error(int code, const char* msg);

// Read-only graph arrays read through the constant address space: uniform indices become scalar
// loads (the compiler cannot otherwise prove they do not alias the inbox being written, and would
// issue vector loads whose waits drain every outstanding row load).
typedef __attribute__((address_space(4))) const int32_t cint32;
__device__ __forceinline__ int32_t sload(const int32_t* p, int i) { return ((cint32*)p)[i]; }

// One workgroup-wide work ticket from an LDS counter (lane 0 takes it, the wave reads it back as a
// scalar). Persistent kernels hand each block's static item share to its waves this way: waves on a
// SIMD issue oldest-first, so equal static per-wave shares leave a CU waiting for its youngest waves.
__device__ __forceinline__ int take_ticket(int* ctr, int lane) {
  int t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(t);
}

// ---------------------------------------------------------------- IB fast path
struct IbFastArgs {
  const uint8_t* in;        // own-order inbox (nullptr for CN pass 0: inputs gathered from ch8)
  uint8_t* out;             // other-order inbox
  const uint8_t* ch8;       // staged channel cluster ids: 4-bit nibbles [N][ldb bytes]
  const int32_t* info;      // per position (heaviest node first): {node, first own-order edge, degree, 0}
  const int32_t* tgt;       // own-order edge -> other-order row
  const int32_t* gather;    // CN pass 0: csr_cols (edge -> variable node); else nullptr
  const uint32_t* img;      // this pass's tables: nt x 64 dwords (256 entries, t*16+m)
  const int32_t* gate;      // kShards flag words that must be non-zero to run (nullptr: run)
  int32_t* unsat;           // kShards flag words to set when a check is unsatisfied (nullptr: no syndrome)
  int32_t fslot[kMaxD + 1]; // per degree: LDS slot of the final (composite) op
  int32_t nt;               // table quads staged in LDS (4 tables each, common.h layout)
  const uint32_t* cimg;     // this pass's column images: ncs x 16 columns x 2 dwords (stage_cols)
  int32_t ncs;              // column images staged after the table quads
  int8_t ccol[kMaxD + 1][4];// per degree: column image of its i-th column-fetched input
  int32_t n_nodes, nchunks, ldb, B, half, match;   // ldb = row stride in BYTES (2 codewords/byte)
  int32_t n_heavy;          // positions [0, n_heavy) have degree > kLightD (item buffer of MAXD rows)
  uint64_t* trace;          // diagnostics (IBL_TRACE_WAVES): per wave {start clock, end clock, items}, else nullptr
  // small-batch kernels (ib_*_small): tasks of up to 64 consecutive same-degree positions of `info`,
  // {first position, count, degree, 0}; a wave item is (task, word), nwords = ceil(B / 8)
  const int32_t* task;
  int32_t n_tasks, nwords;
};

struct IbDecArgs {
  const uint8_t* vin;       // varnode_inbox [E][ldb]
  const uint8_t* ch8;
  const int32_t* start;
  const int32_t* deg;
  const uint32_t* img;      // decision tables for every pass: imax x nt x 64 dwords
  const int32_t* iters;     // device scalar L (pass index of the decision tables)
  void* out;                // user output [N][B]
  int32_t out_dtype, nt, n_nodes, nchunks, ldb, B, aligned;
  const int32_t* info;      // small-batch decision (ib_dec_small): variable work order and its tasks
  const int32_t* task;
  int32_t n_tasks, nwords;
};

// Fused on-chip IB decoder (short codes): a workgroup decodes 8 codewords at a time (one dword of
// 4-bit messages per edge slot, codeword c in nibble c & 7) through ALL iterations with the messages
// in LDS. Edge slots follow the check-node tasks as in FlFusedArgs; the per-pass table images are the
// per-pass kernels' (staged into the table quads at LDS address 0 before every phase).
struct IbFusedArgs {
  const uint32_t* cn_img;   // CN tables, pass p = 0..imax-1: cn_nt quads x 256 dwords each
  const uint32_t* vn_img;   // VN tables, pass k = 0..imax-2
  const uint32_t* dec_img;  // decision tables, pass k = 0..imax-1
  const uint32_t* chT;      // channel nibbles, [group][position] dwords (codewords 8*group .. 8*group+7),
                            // positions in variable-task order (vn_node)
  const int32_t* cn_task;   // per check task: {first slot, count, degree, 0}
  const int32_t* vn_task;   // per variable task: {first position, count, degree, first vn_slot index}
  const int32_t* vn_node;   // variable position -> node
  const int32_t* vn_slot;   // variable task edge k, lane i at [first + k*count + i] -> message slot
  void* out;                // user output [N][B] (out_dtype)
  int32_t* unsat;           // non-null: CN pass j >= 1 ORs "unsatisfied" into unsat[j*kShards + shard]
  const int32_t* dL;        // non-null: re-run to the device stop iteration *dL (skipped if imax-1)
  int32_t cn_fslot[kMaxD + 1], vn_fslot[kMaxD + 1];
  int32_t cn_nt, vn_nt, dec_nt, nreg;   // quads per pass image; nreg = table quads reserved in LDS (per set)
  int32_t dbuf;             // 1: two table sets of nreg quads (phase p reads set p & 1; the next phase's
                            // set is written during the current phase), no raw buffer
  int32_t n_cn_nodes;
  int32_t cn_uni, vn_uni;   // > 0: every task record is {64 t D, min(64, n - 64 t), D, ...} with this D
                            // (single-degree side): computed from t instead of loaded (no scalar-load
                            // wait, which also drains the wave's LDS queue, per task)
  int32_t n_e, n_v, n_cn_tasks, n_vn_tasks, B, imax, half, match, out_dtype, aligned, ngroups;
  int32_t ncw;              // codewords per workgroup: 8, or 4 (half groups, small batches; see ib_fused)
  uint64_t* trace;          // diagnostics (IBL_TRACE_FUSED): block 0's clock at every phase boundary of its
                            // first group, else nullptr
};

// --------------------------------------------------------------- IB generic path
// Reference-exact flat-vector indexing (any T_ch, T_dec <= 256, any degree).
struct IbGenArgs {
  const uint8_t* in;
  uint8_t* out;
  const uint8_t* ch8;
  const int32_t* start;
  const int32_t* deg;
  const int32_t* tgt;
  const int32_t* gather;
  const int32_t* lut;       // flat int32 CN or VN vector
  const int32_t* mt;        // flat matching vector
  const int32_t* gate;
  int32_t* unsat;
  int64_t lut_len, mt_len;
  int32_t pass, Tc, T, CM, VM, match, n_nodes, ldb, B, half;
};

struct IbGenDecArgs {
  const uint8_t* vin;
  const uint8_t* ch8;
  const int32_t* start;
  const int32_t* deg;
  const int32_t* lut;
  const int32_t* iters;
  void* out;
  int64_t lut_len;
  int32_t out_dtype, Tc, T, VM, n_nodes, ldb, B;
};

// ------------------------------------------------------------------- float path
struct FlArgs {
  const void* in;           // own-order inbox (F)
  void* out;                // other-order inbox (F)
  const void* ch;           // staged channel LLRs [N][ldb] (F)
  const int32_t* start;
  const int32_t* deg;
  const int32_t* tgt;
  const int32_t* gate;
  int32_t* unsat;
  double llr_max;
  int32_t n_nodes, nchunks, ldb, B;
  // degree-2 variable fold (check pass; see fl_cn_item): per check kFoldRec ints {pos0, pos1, dst0, dst1,
  // var0, var1, 0, 0} — edge position of up to two folded variables (-1: none), the check-order row of the
  // variable's other edge in fout, the variable (channel row). fold_mode 0: off; 1: a folded edge's output
  // goes to fout only; 2: to fout and to the variable inbox (early stop: any pass may be the last).
  const int32_t* fold;
  void* fout;               // the next check pass's inbox (check order)
  int32_t fold_mode;
  const int32_t* nodes;     // variable pass: node list (the variables not folded), nullptr = 0..n_nodes-1
  // small-batch kernels (fl_*_small): tasks of up to 64 consecutive same-degree positions of `info` (the IB
  // fast path's work orders, {node, start, degree, 0}); a wave item is (task, word of Vec<F>::N codewords)
  const int32_t* info;
  const int32_t* task;
  int32_t n_tasks, nwords;
};

// Fused float decoder: a workgroup keeps Vec<F>::N codewords (one 16-byte slot per edge) entirely
// in LDS for all iterations. Edge slots are numbered per check-node task (up to 64 check nodes of
// one degree, lane = node): edge k of lane i of a task at slot first + k*count + i, so the check
// pass reads and writes contiguous 16-byte slots; the variable pass gathers through vn_slot.
// fused float kernel phase trace (diagnostic builds): words per phase — [0] start clock, [1 + w] wave w's
// done clock, [17 + w] its task count, [33 + w] its first task's body start (ticket and task record
// taken), [49 + w] that body's end
constexpr int kFlTraceWords = 65;
struct FlFusedArgs {
  const void* ch;           // staged channel LLRs [group][variable position] (Vec<F>::T, fl_stage_t)
  const int32_t* cn_task;   // per check task: {first slot, count, degree, 0}
  const int32_t* vn_task;   // per variable task: {first position, count, degree, first vn_slot index}
  const int32_t* vn_node;   // variable position -> node
  const int32_t* vn_slot;   // variable task edge k, lane i at [first + 64k + i] -> message slot
  void* out;                // user output [N][B] (out_dtype)
  int32_t* unsat;           // non-null: CN pass j ORs "unsatisfied" into unsat[(j-1)*kShards + shard]
  const int32_t* dL;        // non-null: re-run to the device stop iteration *dL (skipped if imax-1)
  double llr_max;
  int32_t n_e, n_v, n_cn_tasks, n_vn_tasks, ldb, B, imax, out_dtype, aligned, ngroups;
  int32_t n_vs;             // variable-edge slot indices (vn_slot), each task's rows padded to 64 lanes
  uint64_t* trace;          // diagnostics (IBL_TRACE_FUSED, -DIBL_FUSED_TRACE=1 builds): block 0's clock at
                            // every phase end of its first group, else nullptr
};

struct FlDecArgs {
  const void* vin0;         // ping-pong varnode inboxes, selected by parity of L
  const void* vin1;
  const void* ch;
  const int32_t* start;
  const int32_t* deg;
  const int32_t* iters;
  void* out;
  int32_t out_dtype, n_nodes, nchunks, ldb, B, aligned;
  const int32_t* info;      // small-batch decision (fl_dec_small): variable work order and its tasks
  const int32_t* task;
  int32_t n_tasks, nwords;
};

// launchers (defined in the .hip translation units, called by capi.hip)
hipError_t launch_ib_stage(const void* ch, int dtype, int n, int B, uint8_t* ch8, int ldb, hipStream_t s);
// writes the first ceil(B / 8) words of every row (the rest of a row is padding no output reads)
hipError_t launch_ib_stage4(const void* ch, int dtype, int n, int B, uint8_t* ch4, int ldb_bytes, hipStream_t s);
hipError_t launch_ib_cn_fast(const IbFastArgs& a, int maxd, int grid, int block, size_t lds, hipStream_t s);
hipError_t launch_ib_vn_fast(const IbFastArgs& a, int maxd, int grid, int block, size_t lds, hipStream_t s);
int ib_fast_chunk(int maxd);  // codewords per wave item of the CN/VN kernel for this max degree
hipError_t launch_ib_dec_fast(const IbDecArgs& a, int grid, int block, size_t lds, hipStream_t s);
// small-batch per-pass kernels (B <= a few words): grid from the item count, block kSmallBlock
// IB small-batch kernels: built for blocks of up to 1024 threads, launched with small_block(nwords) threads
constexpr int kSmallBlock = 1024;
// block size by words per row (same box, DVB-S2 i_max = 50, profiles/r05_ib_small_block_ab.json): one word
// (B <= 8) 256 threads — more blocks stage their tables in parallel; up to 8 words 512; more 1024
__host__ __device__ constexpr int small_block(int nwords) { return nwords <= 1 ? 256 : (nwords <= 8 ? 512 : 1024); }
constexpr int kFlSmallBlock = 256;             // float small-batch kernels (the degree-16 BP bodies need > 128 VGPRs)
constexpr int kSmallBatchDefault = 224;   // batches up to this many codewords take the small-batch kernels
constexpr int kFlSmallBatchDefault = 64;  // the float decoders' default threshold
hipError_t launch_ib_cn_small(const IbFastArgs& a, int maxd, int grid, size_t lds, hipStream_t s);
hipError_t launch_ib_vn_small(const IbFastArgs& a, int maxd, int grid, size_t lds, hipStream_t s);
hipError_t launch_ib_dec_small(const IbDecArgs& a, int grid, size_t lds, hipStream_t s);
hipError_t ib_small_private_bytes(int cn_maxd, int vn_maxd, size_t* bytes, const char** name);
hipError_t ib_fast_occupancy(int which, int maxd, int block, size_t lds, int* blocks_per_cu);
// Largest private (scratch) segment over the fast-path kernels a decoder of max degree maxd launches
// (CN with and without gather, VN, decision); *name receives that kernel's name.
hipError_t ib_fast_private_bytes(int cn_maxd, int vn_maxd, size_t* bytes, const char** name);
hipError_t launch_ib_stage_t(const void* ch, int dtype, int n, int B, const int32_t* perm, uint32_t* chT,
                             hipStream_t s);
hipError_t launch_ib_fused(const IbFusedArgs& a, int cmax, int vmax, int grid, int block, size_t lds, hipStream_t s);
hipError_t ib_fused_occupancy(int cmax, int vmax, int ncw, size_t lds, int* blocks_per_cu, int* block,
                              size_t* private_bytes);
hipError_t launch_ib_cn_gen(const IbGenArgs& a, hipStream_t s);
hipError_t launch_ib_vn_gen(const IbGenArgs& a, hipStream_t s);
hipError_t launch_ib_dec_gen(const IbGenDecArgs& a, hipStream_t s);
hipError_t launch_finalize(const int32_t* flags, int imax, int early, int32_t* dL, int32_t* user, hipStream_t s);
// ------------------------------------------------------------ channel generation
constexpr int kMaxT = 64;         // largest channel alphabet of ibl_channel_sample
constexpr int kChBinSh = 43, kChBins = 1 << (53 - kChBinSh);   // binned CDF inversion: 1024 bins of m's 53 bits
struct ChArgs {
  uint64_t kthr[kMaxT + 1]; // floor(cdf[w] * 2^53) of the p(t | x = 0) CDF: u = m 2^-53 > cdf[w] <=> m > kthr[w]
  double llr[kMaxT];        // output_LLRs (LLR outputs)
  uint64_t ctr[4];          // Philox counter before the batch (numpy Philox `counter`)
  uint64_t key[2];          // Philox key (numpy Philox `key`)
  const uint8_t* bits;      // optional [n][B] codeword bits (1 mirrors the cluster), nullptr = all-zero
  void* out;                // [n][ld] u8 / i32 cluster ids or f32 / f64 LLRs
  int64_t total, ld;        // n*B, output row stride (elements)
  int32_t B, T, dtype;
  int32_t sorted;           // kthr[1..T] non-decreasing (every CDF without NaNs): the binned inversion applies
  uint16_t bin[kChBins];    // sorted: per bin of m's top bits, base | n << 8 (channel_kernels.hip invert_binned)
};
hipError_t launch_ch_sample(const ChArgs& a, hipStream_t s);

// ------------------------------------------------------------------ encoder
hipError_t launch_enc_pack(const uint8_t* in, int rows, int B, int Bw, uint32_t* out, hipStream_t s);
hipError_t launch_enc_ax(const uint32_t* x, const int32_t* indptr, const int32_t* cols, int M, int Bw, uint32_t* r,
                         hipStream_t s);
hipError_t launch_enc_subst(const uint32_t* in, uint32_t* out, const int32_t* indptr, const int32_t* cols, int M,
                            int Bw, int dir, hipStream_t s);
hipError_t launch_enc_scan(const uint32_t* r, uint32_t* tot, int M, int Bw, int dir, uint32_t* p, hipStream_t s);
int enc_scan_segments();
hipError_t launch_enc_gather(const uint32_t* in, const int32_t* order, int M, int Bw, uint32_t* out, hipStream_t s);
hipError_t launch_enc_unpack(const uint8_t* info, const uint32_t* p, int K, int M, int B, int Bw, uint8_t* code,
                             hipStream_t s);
hipError_t launch_random_bits(uint64_t seed, uint64_t offset, int64_t total, uint8_t* out, hipStream_t s);
hipError_t launch_count_errors(const void* x, int dtype, int64_t rows, int B, int64_t ld, double thr,
                               const uint8_t* bits, int64_t bits_ld, unsigned long long* cnt, hipStream_t s);

hipError_t launch_count_below(const void* x, int dtype, int64_t rows, int B, int64_t ld, double thr,
                              unsigned long long* cnt, hipStream_t s);

hipError_t launch_fl_send(const FlArgs& a, int prec, hipStream_t s);
// rule: channel-LLR precondition counted into *bad (0 none, 1 NaN, 2 NaN / |x| > ln(DBL_MAX), 3 NaN / inf as fp32;
// float_kernels.hip llr_bad)
hipError_t launch_fl_stage(const void* x, int in_dtype, int n, int B, void* dst, int prec, int ldb, int rule,
                           int32_t* bad, hipStream_t s);
hipError_t launch_fl_stage_t(const void* x, int in_dtype, int n, int B, const int32_t* perm, void* dst, int prec,
                             int rule, int32_t* bad, hipStream_t s);
hipError_t launch_fl_cn(const FlArgs& a, int kind, int prec, int maxd, int grid, hipStream_t s);
hipError_t launch_fl_vn(const FlArgs& a, int prec, int maxd, int grid, hipStream_t s);
int fl_vn_chunk(int prec, int maxd);   // codewords per wave item of the per-pass variable kernel
constexpr int kFlRowPad = 512;   // float inbox rows are padded to this many codewords (every item shape fits)
hipError_t launch_fl_dec(const FlDecArgs& a, int prec, int grid, hipStream_t s);
// small-batch float kernels (B <= a few words; lane = node): kFlSmallBlock threads per block
hipError_t launch_fl_cn_small(const FlArgs& a, int kind, int prec, int maxd, int grid, hipStream_t s);
hipError_t launch_fl_vn_small(const FlArgs& a, int prec, int maxd, int grid, hipStream_t s);
hipError_t launch_fl_dec_small(const FlDecArgs& a, int prec, int grid, hipStream_t s);
hipError_t fl_small_private_bytes(int kind, int prec, int cn_maxd, int vn_maxd, size_t* bytes, const char** name);
hipError_t fl_occupancy(int which, int kind, int prec, int maxd, int* blocks_per_cu);
// Largest private segment over the float kernels of (kind, prec, degrees); fused included when asked.
hipError_t fl_private_bytes(int kind, int prec, int cn_maxd, int vn_maxd, bool fused, size_t* bytes,
                            const char** name);
int fl_block(int which, int kind, int prec, int maxd);  // threads per block of the float CN (0) / VN (1) kernels
hipError_t launch_fl_fused(const FlFusedArgs& a, int kind, int prec, int cmax, int vmax, int grid, size_t lds,
                           hipStream_t s);
hipError_t fl_fused_occupancy(int kind, int prec, int cmax, int vmax, size_t lds, int* blocks_per_cu, int* block);

}  // namespace ibl
