// Batched systematic LDPC encoding on the device — replaces the reference's
// per-codeword host encoder Discrete_LDPC_decoding/LDPC_encoder.py encode (:86-123, GF2MatrixMul
// :164-190) called by AWGN_Channel_Transmission/LDPC_Transmitter.py transmit (:109-125).
//
// Codewords are bit-packed 32 per dword ([row][word], word w = codewords 32w..32w+31), so every
// GF(2) row operation is one XOR per lane for 32 codewords:
//   enc_pack     u8 [K][B] information bits -> [K][Bw] words
//   enc_ax       r = A x: per (check row, word) XOR of the information words of the row
//   enc_subst    p_i = r_i xor XOR_{j in T_i} p_j in substitution order (T strictly triangular): one
//                thread per word walks the rows; the previous row's value rides in a register, other
//                dependencies are re-read (same thread wrote them; agent-scope accesses keep L2 order)
//   enc_gather   r = r[row_order] between the L and P substitutions of the factorised case
//   enc_unpack   [x; p] -> u8 [N][B] codewords
// Plus the BER drivers' helpers: random information bits from the numpy-compatible Philox stream
// (bit = top bit of each 64-bit output) and an error counter against the transmitted bits.
#include "common.h"

namespace ibl {

__global__ void enc_pack(const uint8_t* __restrict__ in, int rows, int B, int Bw, uint32_t* __restrict__ out) {
  const int64_t total = (int64_t)rows * Bw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / Bw;
    const int w = (int)(i - r * Bw);
    uint32_t v = 0;
    const uint8_t* p = in + r * B + 32 * w;
    const int n = min(32, B - 32 * w);
    for (int k = 0; k < n; ++k) v |= (uint32_t)(p[k] & 1) << k;
    out[i] = v;
  }
}

__global__ void enc_ax(const uint32_t* __restrict__ x, const int32_t* __restrict__ indptr,
                       const int32_t* __restrict__ cols, int M, int Bw, uint32_t* __restrict__ r) {
  const int64_t total = (int64_t)M * Bw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / Bw);
    const int w = (int)(i - (int64_t)row * Bw);
    uint32_t v = 0;
    for (int e = indptr[row]; e < indptr[row + 1]; ++e) v ^= x[(int64_t)cols[e] * Bw + w];
    r[i] = v;
  }
}

// rows processed ascending (dir > 0) or descending; in and out may not alias
__global__ void enc_subst(const uint32_t* __restrict__ in, uint32_t* out, const int32_t* __restrict__ indptr,
                          const int32_t* __restrict__ cols, int M, int Bw, int dir) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= Bw) return;
  uint32_t prev = 0;
  int prev_row = -1;
  for (int k = 0; k < M; ++k) {
    const int i = dir > 0 ? k : M - 1 - k;
    uint32_t v = in[(int64_t)i * Bw + w];
    for (int e = indptr[i]; e < indptr[i + 1]; ++e) {
      const int j = cols[e];
      v ^= (j == prev_row) ? prev
                           : __hip_atomic_load(out + (int64_t)j * Bw + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(out + (int64_t)i * Bw + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = v;
    prev_row = i;
  }
}

// Bidiagonal P (p_i = r_i xor p_{i-dir}: the IRA parity of DVB-S2): p is a prefix XOR of r along
// the substitution order, computed as a segmented scan — totals of kEncSeg row segments per word,
// then each segment re-walked from the XOR of the segments before it.
constexpr int kEncSeg = 64;
__global__ void enc_scan_tot(const uint32_t* __restrict__ r, int M, int Bw, int seg_len, int dir,
                             uint32_t* __restrict__ tot) {
  const int64_t total = (int64_t)kEncSeg * Bw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int sg = (int)(i / Bw);
    const int w = (int)(i - (int64_t)sg * Bw);
    uint32_t v = 0;
    for (int k = sg * seg_len; k < min((sg + 1) * seg_len, M); ++k) {
      const int row = dir > 0 ? k : M - 1 - k;
      v ^= r[(int64_t)row * Bw + w];
    }
    tot[i] = v;
  }
}
__global__ void enc_scan_out(const uint32_t* __restrict__ r, const uint32_t* __restrict__ tot, int M, int Bw,
                             int seg_len, int dir, uint32_t* __restrict__ p) {
  const int64_t total = (int64_t)kEncSeg * Bw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int sg = (int)(i / Bw);
    const int w = (int)(i - (int64_t)sg * Bw);
    uint32_t acc = 0;
    for (int t = 0; t < sg; ++t) acc ^= tot[(int64_t)t * Bw + w];
    for (int k = sg * seg_len; k < min((sg + 1) * seg_len, M); ++k) {
      const int row = dir > 0 ? k : M - 1 - k;
      acc ^= r[(int64_t)row * Bw + w];
      p[(int64_t)row * Bw + w] = acc;
    }
  }
}

__global__ void enc_gather(const uint32_t* __restrict__ in, const int32_t* __restrict__ order, int M, int Bw,
                           uint32_t* __restrict__ out) {
  const int64_t total = (int64_t)M * Bw;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(i / Bw);
    const int w = (int)(i - (int64_t)row * Bw);
    out[i] = in[(int64_t)order[row] * Bw + w];
  }
}

__global__ void enc_unpack(const uint8_t* __restrict__ info, const uint32_t* __restrict__ p, int K, int M, int B,
                           int Bw, uint8_t* __restrict__ code) {
  const int64_t total = (int64_t)(K + M) * B;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / B;
    const int c = (int)(i - r * B);
    code[i] = r < K ? (uint8_t)(info[i] & 1) : (uint8_t)((p[(r - K) * Bw + (c >> 5)] >> (c & 31)) & 1u);
  }
}

// ---------------------------------------------------------------- BER-driver helpers
constexpr uint64_t kInfoBitsKeyHi = 1;   // Philox key word 1 of the information-bit stream

__device__ __forceinline__ void philox4x64_10_e(uint64_t c[4], uint64_t k0, uint64_t k1) {
  constexpr uint64_t M0 = 0xD2E7470EE14C6C93ull, M1 = 0xCA5A826395121157ull;
  constexpr uint64_t W0 = 0x9E3779B97F4A7C15ull, W1 = 0xBB67AE8584CAA73Bull;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t hi0 = __umul64hi(M0, c[0]), lo0 = M0 * c[0];
    const uint64_t hi1 = __umul64hi(M1, c[2]), lo1 = M1 * c[2];
    const uint64_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += W0; k1 += W1;
  }
}

// Information bits use Philox key (seed, 1); the channel generator (channel_kernels.hip) uses key
// (seed, 0). The high key word keeps the two streams disjoint for every seed: with one key, the bit
// at a position would be the top bit of the very output whose mantissa is the channel uniform there,
// and the noise would depend on the transmitted bit.
__global__ void random_bits(uint64_t seed, uint64_t offset, int64_t total, uint8_t* out) {
  const int64_t nblk = (total + 3) / 4;
  for (int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; blk < nblk; blk += (int64_t)gridDim.x * blockDim.x) {
    uint64_t c[4] = {offset, 0, 0, 0};
    const uint64_t add = (uint64_t)blk + 1;
    c[0] += add;
    if (c[0] < add) c[1] = 1;
    philox4x64_10_e(c, seed, kInfoBitsKeyHi);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = blk * 4 + s;
      if (i < total) out[i] = (uint8_t)(c[s] >> 63);
    }
  }
}

// -------------------------------------------------------------------- launchers
static int grid_for(int64_t total) { return (int)std::min<int64_t>(std::max<int64_t>((total + 255) / 256, 1), 8192); }

hipError_t launch_enc_pack(const uint8_t* in, int rows, int B, int Bw, uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(enc_pack, dim3(grid_for((int64_t)rows * Bw)), dim3(256), 0, s, in, rows, B, Bw, out);
  return hipGetLastError();
}
hipError_t launch_enc_ax(const uint32_t* x, const int32_t* indptr, const int32_t* cols, int M, int Bw, uint32_t* r,
                         hipStream_t s) {
  hipLaunchKernelGGL(enc_ax, dim3(grid_for((int64_t)M * Bw)), dim3(256), 0, s, x, indptr, cols, M, Bw, r);
  return hipGetLastError();
}
hipError_t launch_enc_subst(const uint32_t* in, uint32_t* out, const int32_t* indptr, const int32_t* cols, int M,
                            int Bw, int dir, hipStream_t s) {
  hipLaunchKernelGGL(enc_subst, dim3((Bw + 63) / 64), dim3(64), 0, s, in, out, indptr, cols, M, Bw, dir);
  return hipGetLastError();
}
hipError_t launch_enc_scan(const uint32_t* r, uint32_t* tot, int M, int Bw, int dir, uint32_t* p, hipStream_t s) {
  const int seg_len = (M + kEncSeg - 1) / kEncSeg;
  const int g = grid_for((int64_t)kEncSeg * Bw);
  hipLaunchKernelGGL(enc_scan_tot, dim3(g), dim3(256), 0, s, r, M, Bw, seg_len, dir, tot);
  hipLaunchKernelGGL(enc_scan_out, dim3(g), dim3(256), 0, s, r, tot, M, Bw, seg_len, dir, p);
  return hipGetLastError();
}
int enc_scan_segments() { return kEncSeg; }
hipError_t launch_enc_gather(const uint32_t* in, const int32_t* order, int M, int Bw, uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(enc_gather, dim3(grid_for((int64_t)M * Bw)), dim3(256), 0, s, in, order, M, Bw, out);
  return hipGetLastError();
}
hipError_t launch_enc_unpack(const uint8_t* info, const uint32_t* p, int K, int M, int B, int Bw, uint8_t* code,
                             hipStream_t s) {
  hipLaunchKernelGGL(enc_unpack, dim3(grid_for((int64_t)(K + M) * B)), dim3(256), 0, s, info, p, K, M, B, Bw, code);
  return hipGetLastError();
}
hipError_t launch_random_bits(uint64_t seed, uint64_t offset, int64_t total, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(random_bits, dim3(grid_for((total + 3) / 4)), dim3(256), 0, s, seed, offset, total, out);
  return hipGetLastError();
}

}  // namespace ibl
