/*
 * ibldpc.h — C ABI of the MI355X-native batched LDPC decoding engine (libibldpc.so).
 *
 * Drop-in boundary for the reference's decoder classes (mx-strk/InformationBottleneckDecodingLDPC,
 * snapshot 2024-10-22).  Each entry point names the reference interface it replaces; the
 * Python classes in informationbottleneckdecodingldpc_amd/ keep the reference's method
 * names and call these through ctypes.
 *
 * Conventions
 *   - return 0 (IBL_OK) or a negative IBL_E* code; the message of the last failure on the
 *     calling thread is returned by ibl_last_error();
 *   - d_* pointers are DEVICE pointers owned by the caller (e.g. torch ROCm tensors'
 *     data_ptr() or hipMalloc); `stream` is a hipStream_t (NULL = default stream);
 *   - decode calls are asynchronous on `stream` and never synchronise the host
 *     (the reference reads the syndrome back every iteration; here the early stop is
 *     decided on the device);
 *   - a handle owns its device tables and scratch, is bound to the device it was created
 *     on and is not thread-safe (as the reference's decoder objects, which own their inboxes);
 *   - arrays are [row][codeword] with row stride B (the reference's received_blocks layout).
 */
#ifndef IBLDPC_H
#define IBLDPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IBL_VERSION 3

enum { IBL_OK = 0, IBL_EINVAL = -1, IBL_EHIP = -2, IBL_ENOMEM = -3, IBL_EUNSUPPORTED = -4 };
enum { IBL_U8 = 1, IBL_I32 = 2, IBL_F32 = 3, IBL_F64 = 4 };
enum { IBL_MINSUM = 0, IBL_BP = 1 };
enum { IBL_PATH_AUTO = 0, IBL_PATH_PASSES = 1, IBL_PATH_FUSED = 2 };
enum { IBL_FLAG_FORCE_GENERIC = 1 };

typedef struct ibl_graph ibl_graph;
typedef struct ibl_ib ibl_ib;
typedef struct ibl_float ibl_float;

int ibl_version(void);
const char* ibl_last_error(void);
/* number of visible HIP devices (0 on a machine without GPU) */
int ibl_device_count(int32_t* n);

/*
 * Tanner-graph index construction on the HOST (no device needed).
 * Replaces map_node_connections (Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py:121-170;
 * regular copy discrete_LDPC_decoder.py:88-130).  Input: canonical CSR of H (column indices
 * strictly ascending within each row).  Outputs (caller-allocated): cn_start[n_c], cn_deg[n_c],
 * tgt_cn[E] (= target_memory_cells_checknodes), vn_start[n_v], vn_deg[n_v],
 * tgt_vn[E] (= target_memory_cells_varnodes).
 */
int ibl_map_node_connections(int32_t n_v, int32_t n_c, const int32_t* csr_indptr, const int32_t* csr_cols,
                             int32_t* cn_start, int32_t* cn_deg, int32_t* tgt_cn,
                             int32_t* vn_start, int32_t* vn_deg, int32_t* tgt_vn);

/*
 * Upload a code graph to `device` (host arrays in, canonical CSR of H).
 * Replaces the index-array upload half of init_OpenCL_decoding
 * (discrete_LDPC_decoder_irreg.py:191-204, min_sum_decoder_irreg.py:182-195).
 */
int ibl_graph_create(int32_t n_v, int32_t n_c, const int32_t* csr_indptr, const int32_t* csr_cols,
                     int32_t device, ibl_graph** out);
int ibl_graph_info(const ibl_graph* g, int32_t* n_v, int32_t* n_c, int64_t* n_e, int32_t* d_c_max,
                   int32_t* d_v_max);
void ibl_graph_destroy(ibl_graph* g);

/*
 * Information-bottleneck (integer lookup-table) decoder.
 * Replaces Discrete_LDPC_Decoder_class_irregular.init_OpenCL_decoding
 * (discrete_LDPC_decoder_irreg.py:172-243) and Discrete_LDPC_Decoder_class.init_OpenCL_decoding
 * (discrete_LDPC_decoder.py:132-200): uploads the CN / VN LUT vectors (reference layout, int32,
 * entries in [0, T_dec)), the matching vectors (irregular class; ignored unless match != 0) and
 * allocates inboxes for up to max_batch codewords (`msg_at_time`).  The CN/VN vector lengths
 * must be at least the reference's (T_ch^2 + (CM-3) T_ch T + (I-1)(CM-2) T^2, resp.
 * I (T_ch T + (VM-1) T^2), CM/VM = the graph's maximum check/variable degree).
 * Fast path (LDS-resident tables) when T_ch == T_dec <= 16 and all degrees <= 16; otherwise a
 * generic reference-indexing path.  flags: IBL_FLAG_FORCE_GENERIC.
 */
int ibl_ib_create(const ibl_graph* g, int32_t T_ch, int32_t T_dec, int32_t imax,
                  const int32_t* cn_lut, int64_t cn_len, const int32_t* vn_lut, int64_t vn_len,
                  const int32_t* match_cn, int64_t mc_len, const int32_t* match_vn, int64_t mv_len,
                  int32_t match, int32_t max_batch, int32_t flags, ibl_ib** out);
/* 1 = LDS fast path, 0 = generic path */
int ibl_ib_path(const ibl_ib* h);
/*
 * Decode path of an IB decoder on the fast path (no reference counterpart; results are identical):
 *   IBL_PATH_AUTO (default)  the fused on-chip kernel when the code fits (E * 4 bytes of messages
 *                            for 8 codewords plus the largest pass's table quads <= 160 KiB,
 *                            check degrees >= 2; e.g. regular (3,6) N=8000, WLAN), else per-pass.
 *                            Tables sit in quads of 4 and the quads in 64-KiB super-regions of two,
 *                            so an odd quad count rounds up (1 quad: 64 KiB, 3 quads: 128 KiB), plus
 *                            1 KiB of raw image per quad: a code whose largest pass needs 3 quads
 *                            (9-12 tables) is fused up to E = 7,420 edges (E * 4 <= 29,680 B), 4
 *                            quads up to 7,164, 1 or 2 quads (<= 8 tables) up to 24,572 / 24,060;
 *                            the per-pass fast path holds at most 4 quads (16 tables) a pass;
 *   IBL_PATH_PASSES          one launch per check / variable pass, messages in HBM;
 *   IBL_PATH_FUSED           the fused kernel (IBL_EUNSUPPORTED if the code does not fit).
 * ibl_ib_path_in_use reports 1 when decodes run the fused kernel.  With the fused kernel the timing
 * API reports each fused launch as one check-node launch.
 */
int ibl_ib_set_path(ibl_ib* h, int32_t path);
int ibl_ib_path_in_use(const ibl_ib* h, int32_t* fused);
/*
 * Small-batch kernels of the fast path (no reference counterpart; outputs identical to the other
 * kernels).  The per-pass fast kernels give every wave one node x 1024 codewords, so a batch of a few
 * codewords — the reference's DVB-S2 driver decodes msg_at_time = 2 (BER_simulation_OpenCL.py:71) —
 * costs what B = 1024 costs; batches B <= max_b instead run kernels whose wave item is up to 64 nodes
 * of one degree (lane = node) x 8 codewords.  Default max_b = 224 (IBL_SMALL_B in the environment when
 * the decoder is created overrides it); 0 turns them off.  The fused on-chip path, when in use, ignores
 * this.  IBL_EUNSUPPORTED if max_b > 0 and the decoder has no fast path.
 */
int ibl_ib_set_small_batch(ibl_ib* h, int32_t max_b);
int ibl_ib_small_batch(const ibl_ib* h, int32_t* max_b);
/*
 * Codewords per workgroup the fused kernel runs a batch of B with (no reference counterpart; results are
 * identical either way): 8, or 4 (half groups) when 2 * ceil(B / 8) workgroups fit the grid or the
 * environment IBL_FUSED_NCW=4 forces them and the half-group kernel fits the device; 0 when decodes do
 * not run the fused kernel.
 */
int ibl_ib_fused_ncw(const ibl_ib* h, int32_t B, int32_t* ncw);
/*
 * Decode B codewords.  Replaces decode_OpenCL (discrete_LDPC_decoder_irreg.py:245-341;
 * discrete_LDPC_decoder.py:202-295).
 *   d_ch   [N][B] channel cluster ids (IBL_U8 or IBL_I32), values in [0, T_ch)
 *   d_out  [N][B] decided cluster ids (IBL_U8 or IBL_I32); bit = (id < T_dec/2)
 *   early_stop  1: stop when the whole batch has zero syndrome (reference behaviour);
 *               0: run exactly imax iterations (benchmark / decode_on_host behaviour)
 *   d_iters     optional device int32 receiving the iteration index used for the output
 *               (the reference's i_num - 1), NULL to skip
 */
int ibl_ib_decode(ibl_ib* h, const void* d_ch, int32_t ch_dtype, int32_t B, void* d_out, int32_t out_dtype,
                  int32_t early_stop, int32_t* d_iters, void* stream);
void ibl_ib_destroy(ibl_ib* h);
/*
 * Kernel timing for the benchmark (no reference counterpart): when enabled, every check-node and
 * variable-node launch of ibl_ib_decode / ibl_float_decode is bracketed by HIP events on the
 * decode stream.  *_read synchronises those events, returns the summed milliseconds and launch
 * counts since the last read (kernels that exited early through the stop flags included), and
 * clears them.
 */
int ibl_ib_timing(ibl_ib* h, int32_t enable);
int ibl_ib_timing_read(ibl_ib* h, double* cn_ms, int32_t* cn_launches, double* vn_ms, int32_t* vn_launches);

/*
 * Float min-sum / belief-propagation decoder.
 * Replaces Min_Sum_Decoder_class_irregular / BeliefPropagationDecoderClassIrregular
 * .init_OpenCL_decoding (min_sum_decoder_irreg.py:167-218, bp_decoder_irreg.py:167-218).
 * kind = IBL_MINSUM | IBL_BP; precision = IBL_F32 (BASELINE build) | IBL_F64 (the reference's
 * double precision); llr_max = clamp of BP / VN messages (the reference's LLR_MAX = 150).
 */
int ibl_float_create(const ibl_graph* g, int32_t kind, int32_t imax, double llr_max, int32_t precision,
                     int32_t max_batch, ibl_float** out);
/*
 * Replaces decode_OpenCL_min_sum (min_sum_decoder_irreg.py:221-287) and
 * decode_OpenCL_belief_propagation (bp_decoder_irreg.py:221-286).
 *   d_llr [N][B] channel LLRs (IBL_F32 / IBL_F64), d_out [N][B] APP LLRs (IBL_F32 / IBL_F64)
 * Precondition: no channel LLR is NaN.  Min-sum allows +-inf (a known bit: every message a variable
 * sends is clamped to +-llr_max, its APP LLR is +-inf), and every message stays finite.  BP box-pluses raw
 * channel values in the first check pass (later box-plus inputs are clamped to +-llr_max): the fp64 decoder
 * (the reference's formula log((1 + e^(a+b)) / (e^a + e^b)), kernels_min_and_BP.cl:5-9) needs
 * |x| <= ln(DBL_MAX) = 709.78 — beyond it e^a overflows and the reference gives NaN; below it an overflowing
 * numerator or vanishing denominator gives +-inf, clamped to +-llr_max as in the reference — and the fp32
 * decoder (an overflow-free form of the same function) needs finite values.  The float kernels take min /
 * max / median as single instructions that assume non-NaN operands: a NaN input gives unspecified outputs.
 */
int ibl_float_decode(ibl_float* h, const void* d_llr, int32_t llr_dtype, int32_t B, void* d_out,
                     int32_t out_dtype, int32_t early_stop, int32_t* d_iters, void* stream);
void ibl_float_destroy(ibl_float* h);
/*
 * Decode path of a float decoder (no reference counterpart; results are identical on both):
 *   IBL_PATH_AUTO (default)  the fused on-chip kernel when the code fits in LDS ((E + N) * 16 bytes of
 *                            messages and channel plus 2 bytes per variable edge slot index — each
 *                            variable task's rows padded to 64 — within 160 KiB, E < 65536, check
 *                            degrees >= 2), else IBL_PATH_PASSES;
 *   IBL_PATH_PASSES          one launch per check / variable pass, messages in HBM;
 *   IBL_PATH_FUSED           the fused kernel (IBL_EUNSUPPORTED if the code does not fit).
 * ibl_float_path_in_use reports 1 when decodes run the fused kernel, 0 otherwise.  With the fused
 * kernel the timing API reports each fused launch as one check-node launch (vn counts stay 0).
 */
int ibl_float_set_path(ibl_float* h, int32_t path);
int ibl_float_path_in_use(const ibl_float* h, int32_t* fused);
/*
 * Degree-2 variable fold of the per-pass path (no reference counterpart; outputs are identical with and
 * without it): the check pass that produces a degree-2 variable's input also computes that variable's
 * output message (clamp(ch + m), kernels_min_and_BP.cl:110-118) into the next check pass's inbox, and the
 * variable pass skips the variable.  *n_folded = number of folded variables (0: off — no degree-2
 * variables, or IBL_FL_FOLD=0 in the environment when the decoder was created).
 */
int ibl_float_folded(const ibl_float* h, int32_t* n_folded);
/*
 * Small-batch kernels of the per-pass float path (no reference counterpart; outputs identical): batches
 * B <= max_b run kernels whose wave item is up to 64 nodes of one degree (lane = node) x 4 fp32 / 2 fp64
 * codewords instead of one node x 256 / 128 codewords; they do not fold.  Default max_b = 64
 * (IBL_SMALL_B at create overrides it); 0 turns them off.  The fused path, when in use, ignores this.
 */
int ibl_float_set_small_batch(ibl_float* h, int32_t max_b);
int ibl_float_small_batch(const ibl_float* h, int32_t* max_b);
/*
 * Channel-LLR precondition check (no reference counterpart).  The staging step of every ibl_float_decode
 * counts the channel LLRs that break ibl_float_decode's precondition — NaN (min-sum); NaN or |x| > 709.78
 * (BP, fp64 decoder); NaN or +-inf (BP, fp32 decoder) — on the device, without a host sync, into one counter
 * per decoder.  This call synchronises the decoder's DEVICE (every stream: the count covers all decodes of
 * this decoder enqueued since the previous call, whatever their stream; `stream` is unused), stores that
 * count in *violations (may be NULL), clears it, and returns IBL_EINVAL (message in ibl_last_error) when it
 * is not 0: the outputs of those decodes are unspecified.  A caller that wants the verdict of one decode
 * calls it once before that decode (to clear) and once after (the reference-named classes do so for every
 * decode that returns host arrays).
 */
int ibl_float_input_check(ibl_float* h, int32_t* violations, void* stream);
int ibl_float_timing(ibl_float* h, int32_t enable);
int ibl_float_timing_read(ibl_float* h, double* cn_ms, int32_t* cn_launches, double* vn_ms, int32_t* vn_launches);

/*
 * Error counter.  Replaces return_errors_all_zero (discrete_LDPC_decoder_irreg.py:343-349,
 * discrete_LDPC_decoder.py:297-300, min_sum_decoder_irreg.py:290-295): counts entries
 * x[r][b] < threshold for r < rows, b < B (row stride ld) into the device int64 *d_count
 * (overwritten).  IB: threshold = T_dec/2; float: threshold = 0.
 */
int ibl_count_below(const void* d_x, int32_t dtype, int64_t rows, int32_t B, int64_t ld, double threshold,
                    int64_t* d_count, void* stream);

/* Channel generation on the device — replaces
 * AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py quantize_direct_OpenCL (:216-240) and
 * quantize_direct_OpenCL_LLR (:242-260) + kernels_quanti_template.cl (:1-52), which sample
 * u ~ U[0,1) with np.random.rand on the host and upload N*B float64 per batch.
 *
 * Writes out[r][b] (row stride ld elements, r < n, b < B) for the quantiser with cluster CDF
 * cdf[0..T] (host array, cdf[0] = 0, T <= 64): t = #{w in 1..T : u > cdf[w]} clamped to T-1,
 * mirrored to T-1-t where d_bits[r*B+b] is 1 (d_bits may be NULL: all-zero codeword).
 * out_dtype IBL_U8 / IBL_I32 store t; IBL_F32 / IBL_F64 store llr[t] (host array of T).
 * u for element i = r*B+b is the i-th output x of numpy's np.random.Philox(counter=offset,
 * key=seed) stream as (x >> 11) * 2^-53; a batch consumes ceil(n*B/4) counter blocks, so the
 * next batch (or GPU) uses offset += ceil(n*B/4).
 */
int ibl_channel_sample(const double* cdf, int32_t T, const double* llr, uint64_t seed, uint64_t offset, int32_t n,
                       int32_t B, const uint8_t* d_bits, void* d_out, int32_t out_dtype, int64_t ld, void* stream);

/* ---- LDPC encoding ------------------------------------------------------
 * Batched systematic encoder, replacing Discrete_LDPC_decoding/LDPC_encoder.py: the plan that
 * getLDPCEncoderParamters (:197-269) derives from H = [A | B] (B triangular with a full diagonal,
 * possibly after reversing its rows -> forward/backward substitution; else GF(2) factorisation
 * gf2factorize :287-340 with its first-candidate pivot rule -> "Matrix Inverse") is built natively
 * from H's canonical CSR (sorted columns); encode (:86-123) / encode_c (:125-162) run for B
 * codewords at once, 32 codewords per dword. A bidiagonal substitution (DVB-S2 IRA parity) runs as a
 * segmented prefix-XOR scan. Returns IBL_EINVAL when B is singular in GF(2) (the reference raises).
 */
typedef struct ibl_encoder ibl_encoder;
int ibl_encoder_create(int32_t n_v, int32_t n_c, const int32_t* indptr, const int32_t* cols, int32_t max_batch,
                       int32_t device, ibl_encoder** out);
/* "Forward Substitution" | "Backward Substitution" | "Matrix Inverse" (EncodingAlgorithm, :269) */
const char* ibl_encoder_algorithm(const ibl_encoder* h);
/* d_info: u8 [K][B] information bits (0/1), d_code: u8 [N][B] codewords [info; parity]
 * (LDPC_Transmitter.py transmit :109-125 encodes msg_at_time columns one by one). */
int ibl_encode(ibl_encoder* h, const uint8_t* d_info, int32_t B, uint8_t* d_code, void* stream);
void ibl_encoder_destroy(ibl_encoder* h);

/* Random information bits u8 [n][B] (np.random.randint(0, 2, (data_len, msg_at_time)) in
 * LDPC_Transmitter.py:111): bit i = top bit of the i-th 64-bit output of numpy's Philox4x64-10
 * stream with key (seed, 1) advanced by `offset` blocks
 * (Generator(Philox(key=seed + 2**64)).advance(offset).random_raw(n*B) >> 63); the next batch uses
 * offset += ceil(n*B/4). Key word 1 = 1 keeps the information bits disjoint from the channel stream
 * of ibl_channel_sample, whose key is (seed, 0), for any seed. */
int ibl_random_bits(uint64_t seed, uint64_t offset, int32_t n, int32_t B, uint8_t* d_out, void* stream);

/* Bit errors of decoder output against transmitted bits: *d_count = #{(r,b): r < rows, b < B,
 * (x[r*ld+b] < threshold) != (bits[r*bits_ld+b] != 0)} as int64 (generalises
 * return_errors_all_zero, Discrete_LDPC_decoding/discrete_LDPC_decoder_irreg.py:343-349, to non-zero codewords;
 * threshold T/2 for cluster ids, 0 for LLRs). x dtype: IBL_U8/IBL_I32/IBL_F32/IBL_F64. */
int ibl_count_errors(const void* d_x, int32_t dtype, int64_t rows, int32_t B, int64_t ld, double threshold,
                     const uint8_t* d_bits, int64_t bits_ld, int64_t* d_count, void* stream);

/* ---- Multi-GPU batch split without torch ------------------------------------------
 * The protocol of informationbottleneckdecodingldpc_amd/distributed.py for C / C++ callers: one process per
 * GPU; rank 0 builds H and the tables and broadcasts them once (ibl_comm_broadcast of the sizes, then of
 * each array — H's CSR and the LUT / matching vectors of ibl_ib_create); every rank decodes its contiguous
 * codeword range (ibl_shard_range) with its own ibl_graph / decoder; per Eb/N0 point one
 * ibl_comm_allreduce_sum_i64 of the counters {errors, bits, codewords}. No collective inside a decode (the
 * reference decodes on one OpenCL device and has no communication, discrete_LDPC_decoder_irreg.py:174-175).
 * Collectives run on RCCL (NCCL's API on ROCm, over xGMI), loaded at run time (dlopen librccl.so.1);
 * IBL_EUNSUPPORTED when it cannot be loaded.
 */
/* [start, start + count) of `rank`'s share of `total` codewords (contiguous, sizes differ by at most 1). */
int ibl_shard_range(int64_t total, int32_t rank, int32_t world, int64_t* start, int64_t* count);
#define IBL_COMM_ID_BYTES 128
typedef struct ibl_comm ibl_comm;
/* rank 0 creates the id (IBL_COMM_ID_BYTES bytes) and hands it to every rank out of band (MPI, a file, TCP) */
int ibl_comm_unique_id(uint8_t* id);
/* collective: every rank of `nranks` calls it with the same id, its rank and its device */
int ibl_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, ibl_comm** out);
/* d_buf: device memory of `bytes` bytes on the communicator's device; asynchronous on `stream` */
int ibl_comm_broadcast(ibl_comm* c, void* d_buf, int64_t bytes, int32_t root, void* stream);
/* in-place sum over ranks of `count` int64 device values; asynchronous on `stream` */
int ibl_comm_allreduce_sum_i64(ibl_comm* c, int64_t* d_buf, int64_t count, void* stream);
void ibl_comm_destroy(ibl_comm* c);

#ifdef __cplusplus
}
#endif

#endif /* IBLDPC_H */
