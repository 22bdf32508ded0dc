// On-device channel generation for the BER drivers.
//
// Replaces AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py quantize_direct_OpenCL (:216-240) and
// quantize_direct_OpenCL_LLR (:242-260) with kernels_quanti_template.cl quantize / quantize_LLR
// (:1-52): the reference draws u ~ U[0,1) with np.random.rand on the host, uploads N*B float64
// per batch, and the kernel maps u to the cluster index by direct inversion of the quantiser's
// CDF p(t | x = 0):  t = #{ w in 1..T : u > cdf[w] }  (then LLR = output_LLRs[t]).
//
// Here the uniforms are generated in the kernel from a counter-based Philox4x64-10 stream, laid
// out exactly like numpy's np.random.Philox(counter=offset, key=seed): element i of the [n][B]
// batch is the stream's i-th 64-bit output (block offset + 1 + i/4, word i%4; numpy increments
// the counter before each block), converted like numpy's random(): (x >> 11) * 2^-53. So any
// batch is reproducible on the host with numpy, and batches / GPUs take disjoint counter ranges.
// Codeword bits of 1 mirror the cluster (t -> T-1-t, quantize_direct :126-143); a t of T (u at or
// above a CDF that sums to slightly less than 1 in floating point, undefined in the reference)
// is clamped to T-1.
#include <algorithm>
#include <climits>
#include <cmath>

#include "common.h"

namespace ibl {

__device__ __forceinline__ void mulhilo64(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
  lo = a * b;
  hi = __umul64hi(a, b);
}

// Philox4x64-10 (Salmon et al., SC'11; Random123 / numpy constants)
__device__ __forceinline__ void philox4x64_10(uint64_t c[4], uint64_t k0, uint64_t k1) {
  constexpr uint64_t M0 = 0xD2E7470EE14C6C93ull, M1 = 0xCA5A826395121157ull;
  constexpr uint64_t W0 = 0x9E3779B97F4A7C15ull, W1 = 0xBB67AE8584CAA73Bull;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint64_t hi0, lo0, hi1, lo1;
    mulhilo64(M0, c[0], hi0, lo0);
    mulhilo64(M1, c[2], hi1, lo1);
    const uint64_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += W0; k1 += W1;
  }
}

// t = #{w in 1..T : u > cdf[w]} on the integers: u = m * 2^-53 with m = x >> 11, and u > cdf[w] <=> m > kthr[w] =
// floor(cdf[w] * 2^53) (the scaling is exact), so the count is 64-bit integer compares — no double conversion
__device__ __forceinline__ int invert_cdf(uint64_t m, const ChArgs& a) {
  int t = 0;
  for (int w = 1; w <= a.T; ++w) t += (m > a.kthr[w]) ? 1 : 0;
  return t < a.T ? t : a.T - 1;
}

// Binned inversion (sorted thresholds, every CDF without NaNs): the host's table (ChArgs::bin, in the kernarg
// segment) gives for bin m >> kChBinSh (the top 10 of m's 53 bits) base = #{w : kthr[w] < bin start} and n =
// #{w : kthr[w] in the bin}, contiguous after base because the thresholds are sorted; t = base + #{k <= n : m >
// kthr[base + k]}. With T thresholds in 1024 bins n is almost always 0: one cached load per sample replaces T
// 64-bit compares. No LDS: the sampler's side-stream slices stay able to co-reside with the decode kernels.
__device__ __forceinline__ int invert_binned(uint64_t m, const ChArgs& a) {
  const uint32_t e = a.bin[(uint32_t)(m >> kChBinSh)];
  const int base = (int)(e & 0xffu), n = (int)(e >> 8);
  int t = base;
  for (int k = 1; k <= n; ++k) t += (m > a.kthr[base + k]) ? 1 : 0;
  return t < a.T ? t : a.T - 1;
}

template <int DT>
__device__ __forceinline__ void ch_put(const ChArgs& a, int64_t o, int t) {
  if constexpr (DT == kU8) reinterpret_cast<uint8_t*>(a.out)[o] = (uint8_t)t;
  else if constexpr (DT == kI32) reinterpret_cast<int32_t*>(a.out)[o] = t;
  else if constexpr (DT == kF32) reinterpret_cast<float*>(a.out)[o] = (float)a.llr[t];
  else reinterpret_cast<double*>(a.out)[o] = a.llr[t];
}

// One Philox block (4 outputs, elements 4 blk .. 4 blk + 3 of the [n][B] batch) per thread and step. Dense rows
// (ld == B, the BER driver's buffers): the 4 elements are consecutive in memory, written as one 4-element store
// when the batch is a multiple of 4 (u8: one dword); otherwise row / column come from one division per block.
template <int DT>
__global__ __launch_bounds__(256) void ch_sample(ChArgs a) {
  const int64_t nblk = (a.total + 3) / 4;
  const bool dense = a.ld == a.B, quad = dense && (a.total & 3) == 0 && !a.bits;
  for (int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; blk < nblk;
       blk += (int64_t)gridDim.x * blockDim.x) {
    // 256-bit counter = offset + 1 + blk (numpy increments before generating)
    uint64_t c[4] = {a.ctr[0], a.ctr[1], a.ctr[2], a.ctr[3]};
    const uint64_t add = (uint64_t)blk + 1;
    c[0] += add;
    uint64_t carry = c[0] < add ? 1 : 0;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      c[i] += carry;
      carry = (carry && c[i] == 0) ? 1 : 0;
    }
    philox4x64_10(c, a.key[0], a.key[1]);
    int t[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) t[s] = a.sorted ? invert_binned(c[s] >> 11, a) : invert_cdf(c[s] >> 11, a);
    const int64_t i0 = blk * 4;
    if (quad) {
      if constexpr (DT == kU8) {
        reinterpret_cast<uint32_t*>(a.out)[blk] = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) |
                                                  ((uint32_t)t[3] << 24);
      } else if constexpr (DT == kI32) {
        reinterpret_cast<int4*>(a.out)[blk] = make_int4(t[0], t[1], t[2], t[3]);
      } else if constexpr (DT == kF32) {
        reinterpret_cast<float4*>(a.out)[blk] = make_float4((float)a.llr[t[0]], (float)a.llr[t[1]], (float)a.llr[t[2]],
                                                            (float)a.llr[t[3]]);
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) ch_put<DT>(a, i0 + s, t[s]);
      }
      continue;
    }
    int64_t r = dense ? 0 : i0 / a.B, col = dense ? i0 : i0 - r * a.B;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = i0 + s;
      if (i >= a.total) break;
      if (col == a.B && !dense) {   // the block crosses into the next row
        ++r;
        col = 0;
      }
      const int tt = (a.bits && a.bits[i]) ? a.T - 1 - t[s] : t[s];
      ch_put<DT>(a, dense ? i : r * a.ld + col, tt);
      ++col;
    }
  }
}

hipError_t launch_ch_sample(const ChArgs& a, hipStream_t s) {
  const int64_t nblk = (a.total + 3) / 4;
  const int grid = (int)std::min<int64_t>((nblk + 255) / 256, 16384);
  const dim3 g(grid > 0 ? grid : 1), b(256);
  switch (a.dtype) {
    case kU8: hipLaunchKernelGGL(ch_sample<kU8>, g, b, 0, s, a); break;
    case kI32: hipLaunchKernelGGL(ch_sample<kI32>, g, b, 0, s, a); break;
    case kF32: hipLaunchKernelGGL(ch_sample<kF32>, g, b, 0, s, a); break;
    default: hipLaunchKernelGGL(ch_sample<kF64>, g, b, 0, s, a); break;
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------ error counters
// return_errors_all_zero (discrete_LDPC_decoder_irreg.py:343-349) and its encoded-codeword generalisation: count
// x[r][b] < thr (a decided 1), or those that differ from the transmitted bits[r][b], over r < rows, b < B. A block
// takes one (row, 256-word segment) item at a time, a lane one 16-byte word of the row (V elements) — so the row /
// column split is one scalar division per item, not one 64-bit division per element as before round 6 — and a wave
// reduces its count into one atomic. Integer outputs compare against ceil(thr) as integers (v < thr <=> v < ceil(thr)).
constexpr int kCntU = 4;   // words per lane and item of the counters

template <typename X>
__device__ __forceinline__ bool cnt_below(X v, double thr, int64_t ilim) {
  if constexpr (sizeof(X) <= 4 && !__is_floating_point(X)) return (int64_t)v < ilim;
  else return (double)v < thr;
}

template <int V>
__device__ __forceinline__ void cnt_load_bits(const uint8_t* p, uint8_t (&b)[V]) {
  if constexpr (V == 16) { const uint4 q = *reinterpret_cast<const uint4*>(p); __builtin_memcpy(b, &q, 16); }
  else if constexpr (V == 4) { const uint32_t q = *reinterpret_cast<const uint32_t*>(p); __builtin_memcpy(b, &q, 4); }
  else if constexpr (V == 2) { const uint16_t q = *reinterpret_cast<const uint16_t*>(p); __builtin_memcpy(b, &q, 2); }
  else b[0] = *p;
}

template <typename X, int V, bool BITS>
__global__ __launch_bounds__(256) void count_rows(const X* x, int64_t rows, int B, int64_t ld, double thr, int64_t ilim,
                                                  const uint8_t* bits, int64_t bits_ld, int64_t nseg,
                                                  unsigned long long* cnt) {
  // an item is (row, segment of kCntU x 256 words): a lane issues its kCntU word loads before it counts any,
  // so a wave keeps kCntU 16-byte loads in flight (one in flight measured 2 TB/s on int32 decisions)
  constexpr int U = kCntU;
  unsigned long long c = 0;
  const int W = B / V;
  const int64_t items = rows * nseg;
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    const int64_t r = it / nseg;
    const int w0 = (int)(it - r * nseg) * (256 * U) + (int)threadIdx.x;
    X v[U][V];
    uint8_t bb[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int w = min(w0 + 256 * u, W - 1);
      if constexpr (V > 1) {
        const uint4 q = *reinterpret_cast<const uint4*>(x + r * ld + (int64_t)w * V);
        __builtin_memcpy(v[u], &q, 16);
      } else {
        v[u][0] = x[r * ld + w];
      }
      if constexpr (BITS) cnt_load_bits<V>(bits + r * bits_ld + (int64_t)w * V, bb[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (w0 + 256 * u >= W) break;
#pragma unroll
      for (int s = 0; s < V; ++s) {
        const bool one = cnt_below(v[u][s], thr, ilim);
        if constexpr (BITS) c += (one != (bb[u][s] != 0)) ? 1ull : 0ull;
        else c += one ? 1ull : 0ull;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

template <typename X, bool BITS>
static hipError_t launch_count_t(const void* xv, int64_t rows, int B, int64_t ld, double thr, const uint8_t* bits,
                                 int64_t bits_ld, unsigned long long* cnt, hipStream_t s) {
  constexpr int V = 16 / sizeof(X);
  const X* x = reinterpret_cast<const X*>(xv);
  const bool vec = (B % V) == 0 && (ld % V) == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0 &&
                   (!BITS || ((bits_ld % V) == 0 && (reinterpret_cast<uintptr_t>(bits) % V) == 0));
  const double ct = std::ceil(thr);
  const int64_t ilim = ct > 4.0e18 ? INT64_MAX : (ct < -4.0e18 ? INT64_MIN : (int64_t)ct);
  const int W = vec ? B / V : B;
  const int64_t nseg = (W + 256 * kCntU - 1) / (256 * kCntU), items = rows * nseg;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(items, 8192));
  if (vec)
    hipLaunchKernelGGL((count_rows<X, V, BITS>), dim3(grid), dim3(256), 0, s, x, rows, B, ld, thr, ilim, bits, bits_ld,
                       nseg, cnt);
  else
    hipLaunchKernelGGL((count_rows<X, 1, BITS>), dim3(grid), dim3(256), 0, s, x, rows, B, ld, thr, ilim, bits, bits_ld,
                       nseg, cnt);
  return hipGetLastError();
}

template <bool BITS>
static hipError_t launch_count(const void* x, int dtype, int64_t rows, int B, int64_t ld, double thr,
                               const uint8_t* bits, int64_t bits_ld, unsigned long long* cnt, hipStream_t s) {
  switch (dtype) {
    case kU8: return launch_count_t<uint8_t, BITS>(x, rows, B, ld, thr, bits, bits_ld, cnt, s);
    case kI32: return launch_count_t<int32_t, BITS>(x, rows, B, ld, thr, bits, bits_ld, cnt, s);
    case kF32: return launch_count_t<float, BITS>(x, rows, B, ld, thr, bits, bits_ld, cnt, s);
    default: return launch_count_t<double, BITS>(x, rows, B, ld, thr, bits, bits_ld, cnt, s);
  }
}

hipError_t launch_count_below(const void* x, int dtype, int64_t rows, int B, int64_t ld, double thr,
                              unsigned long long* cnt, hipStream_t s) {
  return launch_count<false>(x, dtype, rows, B, ld, thr, nullptr, 0, cnt, s);
}
hipError_t launch_count_errors(const void* x, int dtype, int64_t rows, int B, int64_t ld, double thr,
                               const uint8_t* bits, int64_t bits_ld, unsigned long long* cnt, hipStream_t s) {
  return launch_count<true>(x, dtype, rows, B, ld, thr, bits, bits_ld, cnt, s);
}

}  // namespace ibl
