// Microbenchmark: dependent 4-bit table-lookup chains, served by the LDS (ds_read_u8 from a 32-bank
// replicated 8-KiB table image, the decoders' layout) and/or by the vector L1 (global_load_ubyte from a
// 1-KiB table in global memory). Reports lookups per clock per CU at the nominal 2.4 GHz for
// (LDS chains, global chains) per wave in {(8,0), (0,8), (8,2), (8,4), (6,2), (8,8)}.
// build: hipcc --offload-arch=gfx950 -O3 -o lookup_rate lookup_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef __attribute__((address_space(3))) const uint8_t lds8_t;

template <int NL, int NG>
__global__ __launch_bounds__(1024) void chains(const uint8_t* __restrict__ gtab, const uint32_t* __restrict__ img,
                                               int steps, uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint32_t* l32 = reinterpret_cast<uint32_t*>(lds);
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) l32[i] = img[i >> 5];   // 8 KiB: row e = t*16+m, bank lane
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t lane4 = (uint32_t)(lane & 31) << 2;
  uint32_t tl[NL > 0 ? NL : 1], tg[NG > 0 ? NG : 1];
#pragma unroll
  for (int k = 0; k < NL; ++k) tl[k] = (lane + k) & 15;
#pragma unroll
  for (int k = 0; k < NG; ++k) tg[k] = (lane * 3 + k) & 15;
  uint32_t m = (threadIdx.x * 7 + blockIdx.x) & 15;
  for (int s = 0; s < steps; ++s) {
    m = (m + 5) & 15;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      uint32_t x;
      asm("v_lshl_or_b32 %0, %1, 11, %2" : "=v"(x) : "v"(tl[k]), "v"((m << 7) | lane4));
      tl[k] = *(lds8_t*)(size_t)x;
    }
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      uint32_t x;
      asm("v_lshl_or_b32 %0, %1, 4, %2" : "=v"(x) : "v"(tg[k]), "v"(m));
      tg[k] = gtab[x] & 15u;
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) acc += tl[k];
#pragma unroll
  for (int k = 0; k < NG; ++k) acc += tg[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NL, int NG>
void run(const uint8_t* gtab, const uint32_t* img, uint32_t* out, int ncu) {
  const int steps = 4096, block = 1024, grid = ncu;
  auto k = chains<NL, NG>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 8192, 0, gtab, img, 64, out);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 8192, 0, gtab, img, steps, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double lk = (double)grid * block * steps * (NL + NG);
  const double per = lk / (ms * 1e-3) / (ncu * 2.4e9);
  printf("{\"lds_chains\": %d, \"global_chains\": %d, \"ms\": %.3f, \"lookups_per_clk_per_cu\": %.2f, "
         "\"lds_part\": %.2f, \"global_part\": %.2f}\n", NL, NG, ms, per, per * NL / (NL + NG), per * NG / (NL + NG));
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<uint8_t> ht(1024);
  for (int i = 0; i < 1024; ++i) ht[i] = (uint8_t)((i * 37 + 11) & 15);
  std::vector<uint32_t> hi(64);
  for (int i = 0; i < 64; ++i) hi[i] = (uint32_t)((i * 13 + 5) & 15) * 0x01010101u;
  uint8_t* gt;
  uint32_t *img, *out;
  hipMalloc(&gt, 1024);
  hipMalloc(&img, 256);
  hipMalloc(&out, (size_t)ncu * 1024 * 4);
  hipMemcpy(gt, ht.data(), 1024, hipMemcpyHostToDevice);
  hipMemcpy(img, hi.data(), 256, hipMemcpyHostToDevice);
  run<8, 0>(gt, img, out, ncu);
  run<0, 8>(gt, img, out, ncu);
  run<8, 2>(gt, img, out, ncu);
  run<8, 4>(gt, img, out, ncu);
  run<6, 2>(gt, img, out, ncu);
  run<8, 8>(gt, img, out, ncu);
  run<16, 0>(gt, img, out, ncu);
  return 0;
}
