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

__device__ __forceinline__ int invert_cdf(double u, const ChArgs& a) {
  int t = 0;
  for (int w = 1; w <= a.T; ++w) t += (u > a.cdf[w]) ? 1 : 0;
  return t < a.T ? t : a.T - 1;
}

__global__ __launch_bounds__(256) void ch_sample(ChArgs a) {
  const int64_t nblk = (a.total + 3) / 4;
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
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int64_t i = blk * 4 + s;
      if (i >= a.total) break;
      const double u = (double)(c[s] >> 11) * (1.0 / 9007199254740992.0);
      int t = invert_cdf(u, a);
      const int64_t r = i / a.B, col = i - r * a.B;
      if (a.bits && a.bits[i]) t = a.T - 1 - t;
      const int64_t o = r * a.ld + col;
      switch (a.dtype) {
        case kU8: reinterpret_cast<uint8_t*>(a.out)[o] = (uint8_t)t; break;
        case kI32: reinterpret_cast<int32_t*>(a.out)[o] = t; break;
        case kF32: reinterpret_cast<float*>(a.out)[o] = (float)a.llr[t]; break;
        default: reinterpret_cast<double*>(a.out)[o] = a.llr[t]; break;
      }
    }
  }
}

hipError_t launch_ch_sample(const ChArgs& a, hipStream_t s) {
  const int64_t nblk = (a.total + 3) / 4;
  const int grid = (int)std::min<int64_t>((nblk + 255) / 256, 16384);
  hipLaunchKernelGGL(ch_sample, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace ibl
