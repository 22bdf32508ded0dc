/*
 * channel_oracle.c — CPU ORACLE for the on-device channel generator.  TEST INFRASTRUCTURE ONLY
 * (same rules as ib_oracle.c: only tests/, smoke() and bench.py's cpu_baseline leg load it).
 *
 * Restates, for ibl_channel_sample, the reference's direct-inversion sampling
 *   AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py quantize_direct (:126-143) /
 *   quantize_direct_OpenCL(_LLR) (:216-260) + kernels_quanti_template.cl (:1-52):
 *     t = #{ w in 1..T : u > cdf[w] },  LLR = output_LLRs[t],  bit 1 mirrors t -> T-1-t
 * with the uniforms u taken from a Philox4x64-10 stream in numpy's layout
 * (np.random.Philox(counter=offset, key=seed): counter incremented before each 4-word block;
 * u = (x >> 11) * 2^-53 as numpy's random()). Pinning: the Philox words against numpy's
 * Philox bit generator, the inversion rule against the reference's quantize_direct run on
 * seeded np.random uniforms (tests/golden/make_golden_channel.py).
 */
#include <stdint.h>

typedef unsigned __int128 u128;

static void philox4x64_10(uint64_t c[4], uint64_t k0, uint64_t k1) {
  const uint64_t M0 = 0xD2E7470EE14C6C93ull, M1 = 0xCA5A826395121157ull;
  const uint64_t W0 = 0x9E3779B97F4A7C15ull, W1 = 0xBB67AE8584CAA73Bull;
  for (int r = 0; r < 10; ++r) {
    const u128 p0 = (u128)M0 * c[0], p1 = (u128)M1 * c[2];
    const uint64_t hi0 = (uint64_t)(p0 >> 64), lo0 = (uint64_t)p0;
    const uint64_t hi1 = (uint64_t)(p1 >> 64), lo1 = (uint64_t)p1;
    const uint64_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += W0; k1 += W1;
  }
}

/* raw stream: out[i] = i-th 64-bit output of Philox(counter = ctr[0..3], key = key[0..1]) */
void ibo_philox_raw(const uint64_t ctr[4], const uint64_t key[2], int64_t count, uint64_t *out) {
  uint64_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  for (int64_t i = 0; i < count; i += 4) {
    if (++c[0] == 0 && ++c[1] == 0 && ++c[2] == 0) ++c[3];
    uint64_t w[4] = {c[0], c[1], c[2], c[3]};
    philox4x64_10(w, key[0], key[1]);
    for (int s = 0; s < 4 && i + s < count; ++s) out[i + s] = w[s];
  }
}

/* inversion of the cluster CDF for uniforms u (reference rule, t == T clamped to T-1) */
void ibo_invert_cdf(const double *u, int64_t count, const double *cdf, int32_t T, const uint8_t *bits,
                    int32_t *t_out) {
  for (int64_t i = 0; i < count; ++i) {
    int32_t t = 0;
    for (int32_t w = 1; w <= T; ++w) t += (u[i] > cdf[w]) ? 1 : 0;
    if (t > T - 1) t = T - 1;
    if (bits && bits[i]) t = T - 1 - t;
    t_out[i] = t;
  }
}

/* ibl_channel_sample restated: clusters of the [n][B] batch (contiguous) */
void ibo_channel_sample(const double *cdf, int32_t T, uint64_t seed, uint64_t offset, int64_t count,
                        const uint8_t *bits, int32_t *t_out) {
  const uint64_t ctr[4] = {offset, 0, 0, 0}, key[2] = {seed, 0};
  for (int64_t i0 = 0; i0 < count; i0 += 4096) {
    uint64_t raw[4096];
    double u[4096];
    const int64_t m = count - i0 < 4096 ? count - i0 : 4096;
    uint64_t c[4] = {ctr[0] + (uint64_t)(i0 / 4), 0, 0, 0};
    if (c[0] < ctr[0]) c[1] = 1;
    ibo_philox_raw(c, key, m, raw);
    for (int64_t k = 0; k < m; ++k) u[k] = (double)(raw[k] >> 11) * (1.0 / 9007199254740992.0);
    ibo_invert_cdf(u, m, cdf, T, bits ? bits + i0 : 0, t_out + i0);
  }
}
