// Float min-sum / belief-propagation LDPC decoding kernels for MI355X (gfx950).
//
// Replaces Continous_LDPC_Decoding/kernels_min_and_BP.cl (fp64 in the reference):
//   send_channel_values_to_checknode_inbox -> fl_stage + fl_cn (first pass gathers nothing: the
//                                            staged channel rows are scattered by fl_send)
//   checknode_update_minsum (:126-167)    -> fl_cn<MINSUM>
//   checknode_update + boxplus (:5-71)    -> fl_cn<BP>
//   varnode_update (:76-123)              -> fl_vn
//   calc_syndrome (:206-227)              -> fused into fl_cn (parity of its inputs)
//   calc_varnode_output (:170-204)        -> fl_dec
//
// Precision: F = float (the BASELINE's float32 build) or double (strict parity build).
//   * min-sum is computed from (min1, min2, sign product, zero count) of the node's inputs —
//     bit-identical to the reference's sequential sign/min fold, which only selects values;
//   * BP folds are evaluated with prefix sharing in exactly the reference's per-output order
//     (t = boxplus(m_next, t), clamped at every step); fp64 uses the reference's formula
//     log((1+e^{a+b})/(e^a+e^b)), fp32 the overflow-free equivalent
//     sgn(a)sgn(b)min(|a|,|b|) + log1p(e^-|a+b|) - log1p(e^-|a-b|) (the naive form overflows
//     float for a+b > 88);
//   * variable-node sums keep the reference's addition order (channel first, then ascending
//     edges) through prefix sharing, so fp64 sums are bit-identical.
// Each wave item is one node x kChunk codewords; a lane holds 16 bytes of every edge row
// (4 fp32 or 2 fp64 codewords; fp64 items cover 128 codewords).
#include <algorithm>

#include "common.h"

namespace ibl {

// Work-item geometry from the hardware registers and the implicit kernel arguments. This source is built with
// the IEEE mode off (_build.py), an attribute the device libraries do not share, so HIP's threadIdx /
// blockIdx / blockDim / gridDim — calls into them — would stay out-of-line calls in every kernel.
// The grid size is the implicit argument hidden_block_count_x (code object v5: offset 0), in the kernarg
// segment. __builtin_amdgcn_grid_size_x() reads the AQL dispatch packet instead, which lives in the queue's
// ring buffer in host memory: every CU's first wave then waits on a host round trip, ~20 us of every launch
// (round 6: the float small-batch passes took 23-32 us at B = 2, the IB ones 7-9 us).
__device__ __forceinline__ int fl_tid() { return (int)__builtin_amdgcn_workitem_id_x(); }
__device__ __forceinline__ int fl_bid() { return (int)__builtin_amdgcn_workgroup_id_x(); }
__device__ __forceinline__ int fl_bdim() { return (int)__builtin_amdgcn_workgroup_size_x(); }
__device__ __forceinline__ int fl_gdim() {
  return *(cint32*)__builtin_amdgcn_implicitarg_ptr();   // constant address space, as the pointer is
}

template <typename F> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  using T = float4;
  __device__ static float get(const T& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }
  __device__ static void set(T& v, int s, float x) {
    if (s == 0) v.x = x; else if (s == 1) v.y = x; else if (s == 2) v.z = x; else v.w = x;
  }
};
template <> struct Vec<double> {
  static constexpr int N = 2;
  using T = double2;
  __device__ static double get(const T& v, int s) { return s == 0 ? v.x : v.y; }
  __device__ static void set(T& v, int s, double x) { if (s == 0) v.x = x; else v.y = x; }
};

// sign(t) * min(llr_max, sign(t) * t)  (kernels_min_and_BP.cl:69,120) is the clamp of t to
// [-llr_max, llr_max] for every non-NaN t, signed zeros included (sign(+-0) = +-0 gives +-0 back):
// one v_med3_f32 in fp32 instead of the 3 compares, 3 selects, 2 products and a min of the literal
// form. Messages are never NaN (ibldpc.h's precondition), and this source is built with
// -fno-honor-nans and the IEEE mode off (_build.py): min / max / median then take their operands
// directly instead of quieting each through a v_max x, x first.
__device__ __forceinline__ float clampllr(float t, float lm) { return __builtin_amdgcn_fmed3f(t, -lm, lm); }
__device__ __forceinline__ double clampllr(double t, double lm) { return fmin(fmax(t, -lm), lm); }

// sign-bit arithmetic of the min-sum check node
template <typename F> struct Bits;
template <> struct Bits<float> {
  using U = uint32_t;
  static constexpr U kSign = 0x80000000u;
  __device__ static U of(float x) { return __float_as_uint(x); }
  __device__ static float from(U u) { return __uint_as_float(u); }
  // on raw messages: min(|a|, |b|), max(|a|, |b|), median(lo, hi, |x|), min(lo, |x|)
  __device__ static float lo_aa(float a, float b) { return fminf(fabsf(a), fabsf(b)); }
  __device__ static float hi_aa(float a, float b) { return fmaxf(fabsf(a), fabsf(b)); }
  __device__ static float med3_a(float lo, float hi, float x) { return __builtin_amdgcn_fmed3f(lo, hi, fabsf(x)); }
  __device__ static float lo_a(float lo, float x) { return fminf(lo, fabsf(x)); }
  __device__ static float lo(float a, float b) { return fminf(a, b); }
  // the compiler keeps v_and_b32 + v_or_b32 for this (gfx9 VOP3 takes no literal): one v_and_or_b32 with
  // the mask in an SGPR places a sign bit
  __device__ static U and_or(U a, U k, U b) {
    U r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    return r;
  }
  __device__ static U sign_mask() { return __builtin_amdgcn_readfirstlane(kSign); }
};
template <> struct Bits<double> {
  using U = uint64_t;
  static constexpr U kSign = 0x8000000000000000ull;
  __device__ static U of(double x) { return (U)__double_as_longlong(x); }
  __device__ static double from(U u) { return __longlong_as_double((long long)u); }
  // median of (lo <= hi, |x|): max(lo, min(hi, |x|))
  __device__ static double lo_aa(double a, double b) { return fmin(fabs(a), fabs(b)); }
  __device__ static double hi_aa(double a, double b) { return fmax(fabs(a), fabs(b)); }
  __device__ static double med3_a(double lo, double hi, double x) { return fmax(lo, fmin(hi, fabs(x))); }
  __device__ static double lo_a(double lo, double x) { return fmin(lo, fabs(x)); }
  __device__ static double lo(double a, double b) { return fmin(a, b); }
  __device__ static U and_or(U a, U k, U b) { return (a & k) | b; }
  __device__ static U sign_mask() { return kSign; }
};

__device__ __forceinline__ double boxplus(double a, double b, double lm) {
  const double boxp = log((1.0 + exp(a + b)) / (exp(a) + exp(b)));
  return clampllr(boxp, lm);
}
// fp32: |a [+] b| = min(|a|,|b|) + ln(1 + e^-(|a|+|b|)) - ln(1 + e^-||a|-|b||)  (>= 0), sign =
// sgn(a) sgn(b). Evaluated on the hardware base-2 exp/log (v_exp_f32 / v_log_f32, ~1 ulp): no
// range reduction or denormal fix-ups, 4 transcendentals + ~12 VALU per operation. a or b = 0
// gives sum == dif, so the two log terms cancel exactly and the result is 0, as in the reference.
__device__ __forceinline__ float boxplus(float a, float b, float lm) {
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const float aa = fabsf(a), ab = fabsf(b);
  const float mn = fminf(aa, ab);
  const float u = __builtin_amdgcn_exp2f(-(aa + ab) * kLog2e);
  const float v = __builtin_amdgcn_exp2f(-fabsf(aa - ab) * kLog2e);
  float mag = fmaf(kLn2, __builtin_amdgcn_logf(1.f + u) - __builtin_amdgcn_logf(1.f + v), mn);
  mag = __builtin_amdgcn_fmed3f(mag, 0.f, lm);  // rounding may leave -ulp for tiny min; clamp to [0, lm] (:69)
  return ((a < 0.f) != (b < 0.f)) ? -mag : mag;
}

__device__ __forceinline__ bool fl_gate(const int32_t* gate, int lane) {
  if (!gate) return true;
  return __ballot(gate[lane] != 0) != 0ull;
}

// Node bodies work on all N codewords of the lane at once. Output rows of degrees > 8 are stored
// as soon as they are final, so only the D input rows are live in registers (WLAN's degree-11
// variable nodes: 136 -> 85 VGPRs, +14 %); degrees <= 8 keep their outputs and store them together
// at the end of the item, which measured 9 % faster on DVB-S2 (3.21 -> 2.93 ms per VN pass).
// IBL_FL_NT = 1: the per-pass kernels' message / channel rows as nontemporal loads and stores (every row is
// streamed once per pass, far beyond the caches at C5's B = 8192). Same box, two repetitions
// (profiles/r05_c5_nontemporal_ab.json): C5 16.37k / 16.39k cw/s vs 16.17k / 16.18k plain (fl_vn 2.05 vs 2.12 ms).
#ifndef IBL_FL_NT
#define IBL_FL_NT 1
#endif
template <typename F> struct NtVec;
template <> struct NtVec<float> { typedef float T __attribute__((ext_vector_type(4))); };
template <> struct NtVec<double> { typedef double T __attribute__((ext_vector_type(2))); };

// one lane's piece (Vec<F>::N codewords) of a row
template <typename F>
__device__ __forceinline__ void fl_row_load(const F* p, F (&v)[Vec<F>::N]) {
  using V = Vec<F>;
  if constexpr (IBL_FL_NT) {
    const typename NtVec<F>::T r = __builtin_nontemporal_load(reinterpret_cast<const typename NtVec<F>::T*>(p));
#pragma unroll
    for (int s = 0; s < V::N; ++s) v[s] = r[s];
  } else {
    const typename V::T r = *reinterpret_cast<const typename V::T*>(p);
#pragma unroll
    for (int s = 0; s < V::N; ++s) v[s] = V::get(r, s);
  }
}

template <typename F>
__device__ __forceinline__ void fl_store_to(void* base, int ldb, int row, int cw0, const F (&v)[Vec<F>::N]) {
  using V = Vec<F>;
  F* p = reinterpret_cast<F*>(base) + (size_t)row * ldb + cw0;
  if constexpr (IBL_FL_NT) {
    typename NtVec<F>::T o;
#pragma unroll
    for (int s = 0; s < V::N; ++s) o[s] = v[s];
    __builtin_nontemporal_store(o, reinterpret_cast<typename NtVec<F>::T*>(p));
  } else {
    typename V::T o;
#pragma unroll
    for (int s = 0; s < V::N; ++s) V::set(o, s, v[s]);
    *reinterpret_cast<typename V::T*>(p) = o;
  }
}
template <typename F>
__device__ __forceinline__ void fl_store(const FlArgs& a, int row, int cw0, const F (&v)[Vec<F>::N]) {
  fl_store_to<F>(a.out, a.ldb, row, cw0, v);
}

template <typename F, int D>
struct FlOut {
  static constexpr bool kImmediate = D > 8;
  static constexpr int N = Vec<F>::N;
  F v[kImmediate ? 1 : D][N];
  // sink(w, o) stores output w
  template <class Sink>
  __device__ __forceinline__ void put(int w, const F (&o)[N], Sink&& sink) {
    if constexpr (kImmediate) {
      sink(w, o);
    } else {
#pragma unroll
      for (int s = 0; s < N; ++s) v[w][s] = o[s];
    }
  }
  template <class Sink>
  __device__ __forceinline__ void flush(Sink&& sink) {
    if constexpr (!kImmediate) {
#pragma unroll
      for (int w = 0; w < D; ++w) sink(w, v[w]);
    }
  }
};

// XOR of the inputs' sign bits for codeword s. Its sign bit is also
// the syndrome parity of the inputs (calc_syndrome, kernels_min_and_BP.cl:206-227: parity of m < 0):
// a check's inputs are never -0, since the staged channel holds no -0 (fl_stage*, which turn -0 into +0:
// equal values) and a variable's output clamp(ch + sum) is -0 only if every addend is.
template <typename F, int D, int NC>
__device__ __forceinline__ typename Bits<F>::U sign_xor(const F (&m)[D][NC], int s) {
  using Bt = Bits<F>;
  typename Bt::U x = Bt::of(m[0][s]);
#pragma unroll
  for (int j = 1; j < D; ++j) x ^= Bt::of(m[j][s]);
  return x;
}

// Syndrome parity of codeword s's inputs: the sign bit of sign_xor (degrees <= 8); larger degrees keep
// the compare-and-mask form (lane masks in SGPRs), which needs no VGPR beside the 16 inputs.
template <typename F, int D, int NC>
__device__ __forceinline__ bool syndrome_bit(const F (&m)[D][NC], int s) {
  if constexpr (D <= 8) {
    return (sign_xor<F, D>(m, s) >> (8 * sizeof(F) - 1)) != 0;
  } else {
    bool p = false;
#pragma unroll
    for (int j = 0; j < D; ++j) p ^= (m[j][s] < F(0));
    return p;
  }
}

// Check-node body on the inputs m of NC codewords (min-sum or BP); put(w, o) receives output w (any
// order of w). IBL_MS_PS = 0 keeps the (min, second min) form for every degree (A/B).
#ifndef IBL_MS_PS
#define IBL_MS_PS 1
#endif
template <int KIND, typename F, int D, int NC, class Put>
__device__ __forceinline__ void fl_cn_body(const F (&m)[D][NC], F lm, Put&& put) {
  constexpr int N = NC;
  F o[N];
  if constexpr (KIND == 0 && D <= 8 && IBL_MS_PS) {
    // min-sum (kernels_min_and_BP.cl:156-162) with prefix / suffix minima: |out_w| = min over the others =
    // min(P_w, S_{w+1}), P_w = min |m_0..m_{w-1}|, S_j = min |m_j..m_{D-1}| — 3(D-2) v_min (|x| as an input
    // modifier) instead of the running (min, second min) pair plus a compare and a select per output
    // (4D - 2); min only selects, so the outputs are the same bits. Signs: XOR of the others' sign bits
    // (sign_xor ^ own), placed with one v_and_or_b32. A zero input gives every other output +-0 and its own
    // the others' minimum, as the reference's sign(0) = 0 fold; the same tiny-LLR assumption as below.
    using Bt = Bits<F>;
    using U = typename Bt::U;
    const U ks = Bt::sign_mask();
    U sg[N];
#pragma unroll
    for (int s = 0; s < N; ++s) sg[s] = sign_xor<F, D>(m, s);
    auto emit = [&](int w, const F (&mag)[N]) __attribute__((always_inline)) {
#pragma unroll
      for (int s = 0; s < N; ++s) o[s] = Bt::from(Bt::and_or(sg[s] ^ Bt::of(m[w][s]), ks, Bt::of(mag[s])));
      put(w, o);
    };
    if constexpr (D == 2) {
      F a[N], b[N];
#pragma unroll
      for (int s = 0; s < N; ++s) { a[s] = fabs(m[1][s]); b[s] = fabs(m[0][s]); }
      emit(0, a);
      emit(1, b);
    } else {
      F S[D][N], P[N], mg[N];   // S[j] for j = 1..D-2
#pragma unroll
      for (int s = 0; s < N; ++s) S[D - 2][s] = Bt::lo_aa(m[D - 2][s], m[D - 1][s]);
#pragma unroll
      for (int j = D - 3; j >= 1; --j)
#pragma unroll
        for (int s = 0; s < N; ++s) S[j][s] = Bt::lo_a(S[j + 1][s], m[j][s]);
      emit(0, S[1]);
#pragma unroll
      for (int s = 0; s < N; ++s) P[s] = fabs(m[0][s]);
#pragma unroll
      for (int w = 1; w <= D - 2; ++w) {
#pragma unroll
        for (int s = 0; s < N; ++s) mg[s] = w + 1 <= D - 2 ? Bt::lo(P[s], S[w + 1][s]) : Bt::lo_a(P[s], m[D - 1][s]);
        emit(w, mg);
#pragma unroll
        for (int s = 0; s < N; ++s) P[s] = Bt::lo_a(P[s], m[w][s]);
      }
      emit(D - 1, P);
    }
  } else if constexpr (KIND == 0) {
    // min-sum (kernels_min_and_BP.cl:156-162): the fold t = sgn(m t) min(|t|, |m|) over the others of
    // output w only selects values, so |out_w| = min over the others = mn1, or mn2 where |m_w| is the
    // minimum (on a tie mn2 == mn1), and its sign is the XOR of the others' sign bits. A zero input
    // (sign() = 0 kills the reference's fold) makes mn1 = 0, so every other output is +-0 as there; the
    // zero's own output is the others' min. Running (mn1, mn2) with v_min / v_med3 on |m| (abs is an
    // input modifier), signs XORed as bits: ~2.5 VALU per input and 4 per output.
    // Assumption (the only case where the closed form and the fold differ): no product m*t of the fold
    // underflows to 0 (sign(0) = 0 would zero the reference's output). Every message is a sum of channel
    // LLRs and selected messages, so each nonzero one is a multiple of the ulp q of the smallest nonzero
    // |channel LLR|; with that LLR >= 2^-50 (fp32; 2^-450 fp64) every product is >= 2^-146 and none
    // underflows (tests/test_gpu_float.py::test_float32_minsum_tiny_llrs runs that boundary bit-exactly).
    using Bt = Bits<F>;
    using U = typename Bt::U;
    F mn1[N], mn2[N];
    U sg[N];
    const U ks = Bt::sign_mask();
#pragma unroll
    for (int s = 0; s < N; ++s) {
      mn1[s] = Bt::lo_aa(m[0][s], m[1][s]);
      mn2[s] = Bt::hi_aa(m[0][s], m[1][s]);
      sg[s] = sign_xor<F, D>(m, s);
#pragma unroll
      for (int j = 2; j < D; ++j) {
        mn2[s] = Bt::med3_a(mn1[s], mn2[s], m[j][s]);
        mn1[s] = Bt::lo_a(mn1[s], m[j][s]);
      }
    }
#pragma unroll
    for (int w = 0; w < D; ++w) {
#pragma unroll
      for (int s = 0; s < N; ++s) {
        const F mag = (fabs(m[w][s]) == mn1[s]) ? mn2[s] : mn1[s];
        const U sx = sg[s] ^ Bt::of(m[w][s]);
        // degrees > 8 keep the compiler's form: the asm operand copies would push the 16-input body past
        // the 128 VGPRs of a 1024-thread block
        o[s] = Bt::from(D <= 8 ? Bt::and_or(sx, ks, Bt::of(mag)) : (sx & Bt::kSign) | Bt::of(mag));
      }
      put(w, o);
    }
  } else if constexpr (sizeof(F) == 4) {
    // fp32 BP: forward-backward box-plus, 3(D-2) operations instead of the (D-2)(D+3)/2 of the
    // reference's per-output folds (degree 7: 15 vs 25; each costs 4 transcendentals). Box-plus is
    // commutative and associative, and |a [+] b| <= min(|a|,|b|) keeps every partial result inside
    // the clamp for clamped inputs, so only the fp32 rounding differs from the reference order
    // (within the tolerance of tests/test_gpu_float.py; the fp64 build keeps the exact order below).
    F S[D][N], P[N];   // S[j] = m_j [+] ... [+] m_{D-1}, j >= 1
#pragma unroll
    for (int s = 0; s < N; ++s) S[D - 1][s] = m[D - 1][s];
#pragma unroll
    for (int j = D - 2; j >= 1; --j)
#pragma unroll
      for (int s = 0; s < N; ++s) S[j][s] = boxplus(m[j][s], S[j + 1][s], lm);
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(S[1][s], lm);
    put(0, o);
#pragma unroll
    for (int s = 0; s < N; ++s) P[s] = m[0][s];
#pragma unroll
    for (int w = 1; w <= D - 2; ++w) {
#pragma unroll
      for (int s = 0; s < N; ++s) o[s] = clampllr(boxplus(P[s], S[w + 1][s], lm), lm);
      put(w, o);
#pragma unroll
      for (int s = 0; s < N; ++s) P[s] = boxplus(m[w][s], P[s], lm);
    }
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(P[s], lm);
    put(D - 1, o);
  } else {
    // BP sequential box-plus folds with prefix sharing (kernels_min_and_BP.cl:63-69)
    F t[N], P[N];
#pragma unroll
    for (int s = 0; s < N; ++s) t[s] = m[1][s];
#pragma unroll
    for (int j = 2; j < D; ++j)
#pragma unroll
      for (int s = 0; s < N; ++s) t[s] = boxplus(m[j][s], t[s], lm);
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(t[s], lm);
    put(0, o);
#pragma unroll
    for (int s = 0; s < N; ++s) P[s] = m[0][s];
#pragma unroll
    for (int w = 1; w <= D - 2; ++w) {
#pragma unroll
      for (int s = 0; s < N; ++s) t[s] = P[s];
#pragma unroll
      for (int j = w + 1; j < D; ++j)
#pragma unroll
        for (int s = 0; s < N; ++s) t[s] = boxplus(m[j][s], t[s], lm);
#pragma unroll
      for (int s = 0; s < N; ++s) o[s] = clampllr(t[s], lm);
      put(w, o);
#pragma unroll
      for (int s = 0; s < N; ++s) P[s] = boxplus(m[w][s], P[s], lm);
    }
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(P[s], lm);
    put(D - 1, o);
  }
}


// Degree-2 variable fold (FlArgs::fold): a degree-2 variable's update is one add and a clamp per output,
// out(c1) = clamp(ch + m(c2 -> v)) (kernels_min_and_BP.cl:110-118; fl_vn_body<D=2> in the same order), so
// the check that produces m(c2 -> v) writes v's message to c1 itself, straight into the next check pass's
// inbox (fout, double-buffered: this pass never reads what it writes), and the variable pass skips v. Per
// folded variable and codeword that moves 2 channel reads instead of the variable pass's 2 message reads,
// 1 channel read and 2 message writes; the outputs are the same bits.
template <int KIND, typename F, int D>
__device__ __forceinline__ void fl_cn_item(const FlArgs& a, int node, int st, int cw0, bool do_par, int valid,
                                           bool& unsat) {
  using V = Vec<F>;
  constexpr int N = V::N;
  const F* src = reinterpret_cast<const F*>(a.in);
  const F lm = (F)a.llr_max;
  int tg[D];   // output rows, loaded up front as scalars (the stores follow each output)
#pragma unroll
  for (int w = 0; w < D; ++w) tg[w] = sload(a.tgt, st + w);
  F m[D][N];
#pragma unroll
  for (int j = 0; j < D; ++j) fl_row_load<F>(src + (size_t)(st + j) * a.ldb + cw0, m[j]);
  // fold record: wave-uniform (scalar) positions, rows and variables; the channel rows load with the inputs
  int fp0 = -1, fp1 = -1, fd0 = 0, fd1 = 0;
  F c0[N], c1[N];
  if (a.fold_mode) {
    const int* fr = a.fold + (size_t)kFoldRec * node;
    fp0 = sload(fr, 0);
    fp1 = sload(fr, 1);
    fd0 = sload(fr, 2);
    fd1 = sload(fr, 3);
    const F* ch = reinterpret_cast<const F*>(a.ch);
    if (fp0 >= 0) fl_row_load<F>(ch + (size_t)sload(fr, 4) * a.ldb + cw0, c0);
    if (fp1 >= 0) fl_row_load<F>(ch + (size_t)sload(fr, 5) * a.ldb + cw0, c1);
  }
  if (do_par) {
#pragma unroll
    for (int s = 0; s < N; ++s) unsat |= syndrome_bit<F, D>(m, s) && s < valid;
  }
  auto fold_put = [&](int w, const F (&c)[N], int row, const F (&o)[N]) __attribute__((always_inline)) {
    F f[N];
#pragma unroll
    for (int s = 0; s < N; ++s) f[s] = clampllr(c[s] + o[s], lm);
    fl_store_to<F>(a.fout, a.ldb, row, cw0, f);
    if (a.fold_mode == 2) fl_store<F>(a, tg[w], cw0, o);
  };
  auto sink = [&](int w, const F (&o)[N]) __attribute__((always_inline)) {
    if (w == fp0) fold_put(w, c0, fd0, o);
    else if (w == fp1) fold_put(w, c1, fd1, o);
    else fl_store<F>(a, tg[w], cw0, o);
  };
  FlOut<F, D> ob;
  fl_cn_body<KIND, F, D>(m, lm, [&](int w, const F (&o)[N]) __attribute__((always_inline)) { ob.put(w, o, sink); });
  ob.flush(sink);
}

// Variable-node body on channel c and inputs m; put(w, o) receives extrinsic output w.
template <typename F, int D, int NC, class Put>
__device__ __forceinline__ void fl_vn_body(const F (&c)[NC], const F (&m)[D][NC], F lm, Put&& put) {
  constexpr int N = NC;
  F o[N];
  if constexpr (D == 1) {
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(c[s], lm);
    put(0, o);
  } else {
    // t = ch + others in ascending order (kernels_min_and_BP.cl:113-118)
    F t[N], Q[N];
#pragma unroll
    for (int s = 0; s < N; ++s) t[s] = c[s] + m[1][s];
#pragma unroll
    for (int j = 2; j < D; ++j)
#pragma unroll
      for (int s = 0; s < N; ++s) t[s] = t[s] + m[j][s];
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(t[s], lm);
    put(0, o);
#pragma unroll
    for (int s = 0; s < N; ++s) Q[s] = c[s] + m[0][s];
#pragma unroll
    for (int w = 1; w <= D - 2; ++w) {
#pragma unroll
      for (int s = 0; s < N; ++s) t[s] = Q[s];
#pragma unroll
      for (int j = w + 1; j < D; ++j)
#pragma unroll
        for (int s = 0; s < N; ++s) t[s] = t[s] + m[j][s];
#pragma unroll
      for (int s = 0; s < N; ++s) o[s] = clampllr(t[s], lm);
      put(w, o);
#pragma unroll
      for (int s = 0; s < N; ++s) Q[s] = Q[s] + m[w][s];
    }
#pragma unroll
    for (int s = 0; s < N; ++s) o[s] = clampllr(Q[s], lm);
    put(D - 1, o);
  }
}


template <typename F, int D>
__device__ __forceinline__ void fl_vn_item(const FlArgs& a, int node, int st, int cw0) {
  using V = Vec<F>;
  constexpr int N = V::N;
  const F* src = reinterpret_cast<const F*>(a.in);
  const F lm = (F)a.llr_max;
  int tg[D];   // output rows, loaded up front as scalars (the stores follow each output)
#pragma unroll
  for (int w = 0; w < D; ++w) tg[w] = sload(a.tgt, st + w);
  F c[N], m[D][N];
  fl_row_load<F>(reinterpret_cast<const F*>(a.ch) + (size_t)node * a.ldb + cw0, c);
#pragma unroll
  for (int j = 0; j < D; ++j) fl_row_load<F>(src + (size_t)(st + j) * a.ldb + cw0, m[j]);
  auto sink = [&](int w, const F (&o)[N]) __attribute__((always_inline)) { fl_store<F>(a, tg[w], cw0, o); };
  FlOut<F, D> ob;
  fl_vn_body<F, D>(c, m, lm, [&](int w, const F (&o)[N]) __attribute__((always_inline)) { ob.put(w, o, sink); });
  ob.flush(sink);
}

// IBL_FL_VN2 = 1: the per-pass variable items take two adjacent 16-byte pieces of every row per lane (2-KiB row
// segments per wave, the guide's faster gather shape: 5.7-5.8 vs 5.5-5.6 TB/s), outputs stored as computed
#ifndef IBL_FL_VN2
#define IBL_FL_VN2 0
#endif
// lane l takes the pieces at cw0 = chunk base + l*N and cw0 + 64*N: each load / store instruction covers 1 KiB
// contiguous, two instructions a 2-KiB segment
template <typename F, int D>
__device__ __forceinline__ void fl_vn_item2(const FlArgs& a, int node, int st, int cw0) {
  constexpr int N = Vec<F>::N, N2 = 2 * N;
  const F* src = reinterpret_cast<const F*>(a.in);
  const F* ch = reinterpret_cast<const F*>(a.ch);
  const F lm = (F)a.llr_max;
  int tg[D];
#pragma unroll
  for (int w = 0; w < D; ++w) tg[w] = sload(a.tgt, st + w);
  F c[N2], m[D][N2];
  {
    F lo[N], hi[N];
    fl_row_load<F>(ch + (size_t)node * a.ldb + cw0, lo);
    fl_row_load<F>(ch + (size_t)node * a.ldb + cw0 + 64 * N, hi);
#pragma unroll
    for (int s = 0; s < N; ++s) { c[s] = lo[s]; c[N + s] = hi[s]; }
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    F lo[N], hi[N];
    fl_row_load<F>(src + (size_t)(st + j) * a.ldb + cw0, lo);
    fl_row_load<F>(src + (size_t)(st + j) * a.ldb + cw0 + 64 * N, hi);
#pragma unroll
    for (int s = 0; s < N; ++s) { m[j][s] = lo[s]; m[j][N + s] = hi[s]; }
  }
  fl_vn_body<F, D, N2>(c, m, lm, [&](int w, const F (&o)[N2]) __attribute__((always_inline)) {
    F lo[N], hi[N];
#pragma unroll
    for (int s = 0; s < N; ++s) { lo[s] = o[s]; hi[s] = o[N + s]; }
    fl_store_to<F>(a.out, a.ldb, tg[w], cw0, lo);
    fl_store_to<F>(a.out, a.ldb, tg[w], cw0 + 64 * N, hi);
  });
}
// (the degree > 8 bodies keep one piece per lane: two would spill)
template <int MAXD>
constexpr bool fl_vn_wide() { return IBL_FL_VN2 && MAXD <= 8; }
int fl_vn_chunk(int prec, int maxd) { return 64 * (prec == kF32 ? 4 : 2) * ((IBL_FL_VN2 && maxd <= 8) ? 2 : 1); }

#define FL_DEG_CASES(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)

// MAXD = largest degree with a body in the switch (8 or 16): the registers of the degree-16 bodies
// would cap every launch's occupancy, so codes with degrees <= 8 get their own instantiation.
// 1024-thread blocks so a CU's waves share one work counter, except where the body needs more than
// the 128 VGPRs such a block allows: the box-plus check node at MAXD=16 or in fp64, and the per-pass
// fp32 min-sum check node at MAXD=16 (512 threads). The fused kernel keeps 1024 threads (its min-sum
// MAXD=16 body fits in 128 VGPRs; 16 waves share the phases).
template <int WHICH, int MAXD, int KIND = 0, typename F = float>
constexpr int fl_block_of() {
  return (WHICH == 0 && ((KIND == 1 && (MAXD > 8 || sizeof(F) == 8)) || (KIND == 0 && MAXD > 8 && sizeof(F) == 4)))
             ? 512 : 1024;
}
// fused kernel: 1024 threads (16 waves share the phases) unless the check bodies need more than 128 VGPRs
// (check degree > 8, or fp64 box-plus)
template <int CMAX, int KIND, typename F>
constexpr int fl_fused_block_of() {
  return (CMAX > 8 || (KIND == 1 && sizeof(F) == 8)) ? 512 : 1024;
}
static int fl_fused_block(int kind, int prec, int cmax) {
  return (cmax > 8 || (kind == 1 && prec == kF64)) ? 512 : 1024;
}

// Items (node, chunk) are dealt to blocks round-robin ({b*wpb + w + nw*i}) and handed to the
// block's waves by LDS tickets (take_ticket): ticket k -> item b*wpb + k % wpb + nw * (k / wpb).
__device__ __forceinline__ int fl_next_item(int* ctr, int lane, int wpb, int nw) {
  const int k = take_ticket(ctr, lane);
  return (int)fl_bid() * wpb + (k % wpb) + nw * (k / wpb);
}

template <int KIND, typename F, int MAXD>
__global__ __launch_bounds__((fl_block_of<0, MAXD, KIND, F>())) void fl_cn(FlArgs a) {
  const int lane = fl_tid() & 63;
  if (!fl_gate(a.gate, lane)) return;
  constexpr int CWL = Vec<F>::N;
  constexpr int CH = 64 * CWL;
  const bool do_par = a.unsat != nullptr;
  bool unsat = false;
  __shared__ int ctr;
  if (fl_tid() == 0) ctr = 0;
  __syncthreads();
  const int wpb = fl_bdim() >> 6, nw = fl_gdim() * wpb, nitems = a.n_nodes * a.nchunks;
  for (;;) {
    const int item = fl_next_item(&ctr, lane, wpb, nw);
    if (item >= nitems) break;
    const int node = __builtin_amdgcn_readfirstlane(item / a.nchunks);
    const int chunk = __builtin_amdgcn_readfirstlane(item - node * a.nchunks);
    const int d = sload(a.deg, node), st = sload(a.start, node);
    const int cw0 = chunk * CH + lane * CWL;
    const int valid = a.B - cw0;
    switch (d) {
#define X(D) case D: if constexpr (D <= MAXD) fl_cn_item<KIND, F, D>(a, node, st, cw0, do_par, valid, unsat); break;
      FL_DEG_CASES(X)
#undef X
      default: break;
    }
  }
  if (do_par && __ballot(unsat) != 0ull && lane == 0)
    atomicOr(&a.unsat[(fl_bid() * wpb + (fl_tid() >> 6)) & (kShards - 1)], 1);
}

template <typename F, int MAXD>
__global__ __launch_bounds__((fl_block_of<1, MAXD>())) void fl_vn(FlArgs a) {
  const int lane = fl_tid() & 63;
  if (!fl_gate(a.gate, lane)) return;
  constexpr int CWL = Vec<F>::N * (fl_vn_wide<MAXD>() ? 2 : 1);
  constexpr int CH = 64 * CWL;
  __shared__ int ctr;
  if (fl_tid() == 0) ctr = 0;
  __syncthreads();
  const int wpb = fl_bdim() >> 6, nw = fl_gdim() * wpb, nitems = a.n_nodes * a.nchunks;
  for (;;) {
    const int item = fl_next_item(&ctr, lane, wpb, nw);
    if (item >= nitems) break;
    const int pos = __builtin_amdgcn_readfirstlane(item / a.nchunks);
    const int chunk = __builtin_amdgcn_readfirstlane(item - pos * a.nchunks);
    const int node = a.nodes ? sload(a.nodes, pos) : pos;   // the fold's variable list skips folded nodes
    const int d = sload(a.deg, node), st = sload(a.start, node);
    const int cw0 = chunk * CH + lane * Vec<F>::N;   // (wide items: the second piece 64 * N further)
    if constexpr (fl_vn_wide<MAXD>()) {
      switch (d) {
        case 1: fl_vn_item2<F, 1>(a, node, st, cw0); break;
#define X(D) case D: if constexpr (D <= MAXD) fl_vn_item2<F, D>(a, node, st, cw0); break;
        FL_DEG_CASES(X)
#undef X
        default: break;
      }
    } else {
      switch (d) {
        case 1: fl_vn_item<F, 1>(a, node, st, cw0); break;
#define X(D) case D: if constexpr (D <= MAXD) fl_vn_item<F, D>(a, node, st, cw0); break;
        FL_DEG_CASES(X)
#undef X
        default: break;
      }
    }
  }
}

// APP LLR = ch + sum of all inputs in ascending order, unclamped (kernels_min_and_BP.cl:196-202).
// Wave item = (node, chunk of 64*N codewords); vector loads of every edge row, vector stores when the
// user buffer is aligned (scalar tail otherwise).
template <typename F>
__global__ __launch_bounds__(256) void fl_dec(FlDecArgs a) {
  using V = Vec<F>;
  constexpr int N = V::N, CH = 64 * N;
  const int L = __builtin_amdgcn_readfirstlane(*a.iters);
  const F* vin = reinterpret_cast<const F*>((L & 1) ? a.vin1 : a.vin0);
  const F* ch = reinterpret_cast<const F*>(a.ch);
  const int lane = fl_tid() & 63;
  const int gw = fl_bid() * (fl_bdim() >> 6) + (fl_tid() >> 6), nw = fl_gdim() * (fl_bdim() >> 6);
  const int nitems = a.n_nodes * a.nchunks;
  for (int item = gw; item < nitems; item += nw) {
    const int n = __builtin_amdgcn_readfirstlane(item / a.nchunks);
    const int chunk = __builtin_amdgcn_readfirstlane(item - n * a.nchunks);
    const int cw0 = chunk * CH + lane * N;
    if (cw0 >= a.B) continue;
    const int d = sload(a.deg, n), st = sload(a.start, n);
    F x[N];
    {
      const typename V::T r = *reinterpret_cast<const typename V::T*>(ch + (size_t)n * a.ldb + cw0);
#pragma unroll
      for (int s = 0; s < N; ++s) x[s] = V::get(r, s);
    }
    if (L > 0)
      for (int v = 0; v < d; ++v) {
        const typename V::T r = *reinterpret_cast<const typename V::T*>(vin + (size_t)(st + v) * a.ldb + cw0);
#pragma unroll
        for (int s = 0; s < N; ++s) x[s] = x[s] + V::get(r, s);
      }
    const size_t o = (size_t)n * a.B + cw0;
    if (a.out_dtype == kF32) {
      float* p = reinterpret_cast<float*>(a.out) + o;
      if (a.aligned && cw0 + N <= a.B) {
        if constexpr (N == 4) *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
        else *reinterpret_cast<float2*>(p) = make_float2((float)x[0], (float)x[1]);
      } else {
#pragma unroll
        for (int s = 0; s < N; ++s)
          if (cw0 + s < a.B) p[s] = (float)x[s];
      }
    } else {
      double* p = reinterpret_cast<double*>(a.out) + o;
      if (a.aligned && cw0 + N <= a.B && N == 2) {
        *reinterpret_cast<double2*>(p) = make_double2((double)x[0], (double)x[1]);
      } else {
#pragma unroll
        for (int s = 0; s < N; ++s)
          if (cw0 + s < a.B) p[s] = (double)x[s];
      }
    }
  }
}

// Channel-LLR precondition (ibldpc.h, ibl_float_input_check), on the bit pattern of the caller's value (this
// source is built with -fno-honor-nans, under which a float compare may be folded as if NaN did not exist):
//   rule 0 checks nothing; rule 1 (min-sum) flags NaN;
//   rule 2 (BP, fp64 decoder) flags NaN and |x| > ln(DBL_MAX) = 709.782712893384: the reference's box-plus
//     log((1 + e^(a+b)) / (e^a + e^b)) (kernels_min_and_BP.cl:5-9) is NaN only once e^a itself overflows —
//     below that an infinite numerator or a zero denominator gives +-inf, which the clamp maps to +-llr_max;
//   rule 3 (BP, fp32 decoder) flags NaN and +-inf of the value the decoder stages (a caller f64 beyond FLT_MAX
//     rounds to inf): the fp32 box-plus (boxplus(float, ...)) is overflow-free for every finite input.
__device__ __forceinline__ bool llr_bad(double x, int rule) {
  const uint64_t u = (uint64_t)__double_as_longlong(x) & 0x7fffffffffffffffull;
  if (rule == 3) return ((uint32_t)__float_as_uint((float)x) & 0x7fffffffu) >= 0x7f800000u;
  return rule != 0 && u > (rule == 2 ? 0x40862e42fefa39efull : 0x7ff0000000000000ull);
}
__device__ __forceinline__ bool llr_bad(float x, int rule) {
  const uint32_t u = __float_as_uint(x) & 0x7fffffffu;
  if (rule == 2) return llr_bad((double)x, 2);
  return rule != 0 && u >= (rule == 3 ? 0x7f800000u : 0x7f800001u);
}
// violations counted per lane (rare path: the check itself is one compare per value)
__device__ __forceinline__ void llr_count(int32_t* bad, int nb) {
  if (nb) atomicAdd(bad, nb);
}

// channel staging: user LLRs (f32/f64, [N][B]) -> F [N][ldb], zero padded, -0 stored as +0; counts inputs that
// violate the precondition of `rule` into *bad
template <typename F>
__global__ void fl_stage(const void* x, int in_dtype, int n, int B, F* dst, int ldb, int rule, int32_t* bad) {
  const size_t total = (size_t)n * ldb;
  int nb = 0;
  for (size_t i = (size_t)fl_bid() * fl_bdim() + fl_tid(); i < total; i += (size_t)fl_gdim() * fl_bdim()) {
    const int row = (int)(i / ldb);
    const int b = (int)(i - (size_t)row * ldb);
    F v = F(0);
    if (b < B) {
      const size_t k = (size_t)row * B + b;
      if (in_dtype == kF32) {
        const float xv = reinterpret_cast<const float*>(x)[k];
        nb += llr_bad(xv, rule);
        v = (F)xv;
      } else {
        const double xv = reinterpret_cast<const double*>(x)[k];
        nb += llr_bad(xv, rule);
        v = (F)xv;
      }
    }
    dst[i] = v + F(0);   // -0 -> +0 (equal values; see sign_xor)
  }
  llr_count(bad, nb);
}

// channel staging for the fused decoder: user LLRs [N][B] -> [group][variable position] 16-byte slots
// (Vec<F>::N codewords of variable perm[pos]), zero padded past B. A slot is N consecutive codewords of
// one row, so each cell is ONE 16-byte load (rows read along the codewords, 512 B per row and tile) and
// the LDS tile only transposes whole cells: 64 positions x 32 groups, rows padded by one cell (the
// position-major reads of a ds_read_b128 lane group then hit 16 distinct 4-bank groups); the slots are
// written along the positions (1 KiB per wave). Non-vector inputs (other dtype, B % N != 0, unaligned)
// load element by element.
template <typename F>
__global__ __launch_bounds__(256) void fl_stage_t(const void* x, int in_dtype, int n, int B, const int32_t* perm,
                                                  typename Vec<F>::T* dst, int rule, int32_t* bad) {
  using V = Vec<F>;
  using VT = typename V::T;
  constexpr int N = V::N, P = 64, G = 32, RW = G + 1;
  __shared__ VT tile[P * RW];
  const int ngroups = (B + N - 1) / N;
  const int ptiles = (n + P - 1) / P, gtiles = (ngroups + G - 1) / G;
  const int own = sizeof(F) == 4 ? kF32 : kF64;
  const bool vec = in_dtype == own && (B % N) == 0 && (reinterpret_cast<uintptr_t>(x) % sizeof(VT)) == 0;
  for (int t = fl_bid(); t < ptiles * gtiles; t += fl_gdim()) {
    const int p0 = (t % ptiles) * P, g0 = (t / ptiles) * G;
    __syncthreads();
    constexpr int kPer = P * G / 256;   // cells per thread, all loads issued before the LDS stores
    VT v[kPer];
    int nb = 0;
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int i = fl_tid() + it * 256;
      const int r = i / G, c = i - r * G;
      const int p = p0 + r, g = g0 + c;
#pragma unroll
      for (int s = 0; s < N; ++s) V::set(v[it], s, F(0));
      if (p < n && g < ngroups) {
        const size_t k = (size_t)perm[p] * B + (size_t)g * N;
        if (vec) {
          v[it] = *reinterpret_cast<const VT*>(reinterpret_cast<const F*>(x) + k);
#pragma unroll
          for (int s = 0; s < N; ++s) nb += llr_bad(V::get(v[it], s), rule);
        } else {
#pragma unroll
          for (int s = 0; s < N; ++s)
            if (g * N + s < B) {
              if (in_dtype == kF32) {
                const float xv = reinterpret_cast<const float*>(x)[k + s];
                nb += llr_bad(xv, rule);
                V::set(v[it], s, (F)xv);
              } else {
                const double xv = reinterpret_cast<const double*>(x)[k + s];
                nb += llr_bad(xv, rule);
                V::set(v[it], s, (F)xv);
              }
            }
        }
      }
    }
    llr_count(bad, nb);
#pragma unroll
    for (int it = 0; it < kPer; ++it) {
      const int i = fl_tid() + it * 256;
      const int r = i / G, c = i - r * G;
      VT o;
#pragma unroll
      for (int s = 0; s < N; ++s) V::set(o, s, V::get(v[it], s) + F(0));   // -0 -> +0 (see sign_xor)
      tile[r * RW + c] = o;
    }
    __syncthreads();
    for (int i = fl_tid(); i < P * G; i += fl_bdim()) {
      const int g = i / P, p = i - g * P;
      if (p0 + p < n && g0 + g < ngroups) dst[(size_t)(g0 + g) * n + p0 + p] = tile[p * RW + g];
    }
  }
}

// send_channel_values_to_checknode_inbox (kernels_min_and_BP.cl:12-29): scatter staged rows
template <typename F>
__global__ void fl_send(FlArgs a) {
  const F* ch = reinterpret_cast<const F*>(a.ch);
  F* dst = reinterpret_cast<F*>(a.out);
  const int per = a.ldb / 4;
  const size_t total = (size_t)a.n_nodes * per;
  for (size_t i = (size_t)fl_bid() * fl_bdim() + fl_tid(); i < total; i += (size_t)fl_gdim() * fl_bdim()) {
    const int n = (int)(i / per);
    const int b4 = (int)(i - (size_t)n * per) * 4;
    if (b4 >= a.B) continue;
    const int d = a.deg[n], st = a.start[n];
    F v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s] = ch[(size_t)n * a.ldb + b4 + s];
    for (int w = 0; w < d; ++w) {
      F* p = dst + (size_t)a.tgt[st + w] * a.ldb + b4;
#pragma unroll
      for (int s = 0; s < 4; ++s) p[s] = v[s];
    }
  }
}

// ------------------------------------------------------- small-batch per-pass kernels
// As the IB small-batch kernels (ib_kernels.hip): the per-pass kernels' wave item is one node x 64 lanes x
// Vec<F>::N codewords, so a batch of 2 costs a pass what B = 256 costs. For small batches a wave item is
// (task, word): up to 64 consecutive same-degree positions of the work order (lane = node) x one word of
// Vec<F>::N codewords, each lane gathering its node's 16-byte pieces of its rows. The node bodies are the
// per-pass kernels' (fl_cn_body / fl_vn_body on the lane's N codewords, same operations in the same order),
// so outputs equal the per-pass path's bit for bit. No fold (the small path runs every variable update).
// A task record {first position, count, degree, contiguous} with contiguous = st0 + 1 says its nodes are
// consecutive with edges st0 + k·d (every DVB-S2 task; plan.h order_tasks): the lane's first edge then needs
// no load and its node (NODE: variable passes) one scalar load per task, as in the IB small-batch kernels.
template <bool NODE, class Args, class Body>
__device__ __forceinline__ void fl_small_items(const Args& a, int lane, Body&& body) {
  const int wpb = fl_bdim() >> 6;
  const int gw = __builtin_amdgcn_readfirstlane(fl_bid() * wpb + (fl_tid() >> 6));
  const int nw = fl_gdim() * wpb, nitems = a.n_tasks * a.nwords;
  for (int item = gw; item < nitems; item += nw) {
    const int t = __builtin_amdgcn_readfirstlane(item / a.nwords);
    const int c = __builtin_amdgcn_readfirstlane(item - t * a.nwords);
    const int p0 = sload(a.task, 4 * t), cnt = sload(a.task, 4 * t + 1), d = sload(a.task, 4 * t + 2);
    const int st1 = sload(a.task, 4 * t + 3);
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

template <typename F>
__device__ __forceinline__ void fl_load_piece(const void* base, int ldb, int row, int cw0, F (&v)[Vec<F>::N]) {
  using V = Vec<F>;
  const typename V::T r = *reinterpret_cast<const typename V::T*>(reinterpret_cast<const F*>(base) + (size_t)row * ldb + cw0);
#pragma unroll
  for (int s = 0; s < V::N; ++s) v[s] = V::get(r, s);
}

template <int KIND, typename F, int D>
__device__ __forceinline__ void fl_cn_small_item(const FlArgs& a, int st, int cw0, bool do_par, bool& unsat) {
  const F lm = (F)a.llr_max;
  int tg[D];
  F m[D][Vec<F>::N];
#pragma unroll
  for (int j = 0; j < D; ++j) {
    tg[j] = a.tgt[st + j];
    fl_load_piece<F>(a.in, a.ldb, st + j, cw0, m[j]);
  }
  if (do_par) {
    const int valid = a.B - cw0;
#pragma unroll
    for (int s = 0; s < Vec<F>::N; ++s) unsat |= syndrome_bit<F, D>(m, s) && s < valid;
  }
  fl_cn_body<KIND, F, D>(m, lm, [&](int w, const F (&o)[Vec<F>::N]) __attribute__((always_inline)) {
    fl_store_to<F>(a.out, a.ldb, tg[w], cw0, o);
  });
}

template <typename F, int D>
__device__ __forceinline__ void fl_vn_small_item(const FlArgs& a, int node, int st, int cw0) {
  const F lm = (F)a.llr_max;
  int tg[D];
  F c[Vec<F>::N], m[D][Vec<F>::N];
  fl_load_piece<F>(a.ch, a.ldb, node, cw0, c);
#pragma unroll
  for (int j = 0; j < D; ++j) {
    tg[j] = a.tgt[st + j];
    fl_load_piece<F>(a.in, a.ldb, st + j, cw0, m[j]);
  }
  fl_vn_body<F, D>(c, m, lm, [&](int w, const F (&o)[Vec<F>::N]) __attribute__((always_inline)) {
    fl_store_to<F>(a.out, a.ldb, tg[w], cw0, o);
  });
}

template <int KIND, typename F, int MAXD>
__global__ __launch_bounds__(kFlSmallBlock) void fl_cn_small(FlArgs a) {
  const int lane = fl_tid() & 63;
  if (!fl_gate(a.gate, lane)) return;
  const bool do_par = a.unsat != nullptr;
  bool unsat = false;
  fl_small_items<false>(a, lane, [&](int, int st, int c, int d) __attribute__((always_inline)) {
    const int cw0 = c * Vec<F>::N;
    switch (d) {
#define X(D) case D: if constexpr (D <= MAXD) fl_cn_small_item<KIND, F, D>(a, st, cw0, do_par, unsat); break;
      FL_DEG_CASES(X)
#undef X
      default: break;
    }
  });
  if (do_par && __ballot(unsat) != 0ull && lane == 0)
    atomicOr(&a.unsat[(fl_bid() * (fl_bdim() >> 6) + (fl_tid() >> 6)) & (kShards - 1)], 1);
}

template <typename F, int MAXD>
__global__ __launch_bounds__(kFlSmallBlock) void fl_vn_small(FlArgs a) {
  const int lane = fl_tid() & 63;
  if (!fl_gate(a.gate, lane)) return;
  fl_small_items<true>(a, lane, [&](int node, int st, int c, int d) __attribute__((always_inline)) {
    const int cw0 = c * Vec<F>::N;
    switch (d) {
      case 1: fl_vn_small_item<F, 1>(a, node, st, cw0); break;
#define X(D) case D: if constexpr (D <= MAXD) fl_vn_small_item<F, D>(a, node, st, cw0); break;
      FL_DEG_CASES(X)
#undef X
      default: break;
    }
  });
}

// APP LLR of the small path: ch + every input in ascending edge order, unclamped (as fl_dec)
template <typename F>
__global__ __launch_bounds__(kFlSmallBlock) void fl_dec_small(FlDecArgs a) {
  const int L = __builtin_amdgcn_readfirstlane(*a.iters);
  const void* vin = (L & 1) ? a.vin1 : a.vin0;
  const int lane = fl_tid() & 63;
  fl_small_items<true>(a, lane, [&](int node, int st, int c, int d) __attribute__((always_inline)) {
    const int cw0 = c * Vec<F>::N;
    F x[Vec<F>::N], r[Vec<F>::N];
    fl_load_piece<F>(a.ch, a.ldb, node, cw0, x);
    if (L > 0)
      for (int v = 0; v < d; ++v) {
        fl_load_piece<F>(vin, a.ldb, st + v, cw0, r);
#pragma unroll
        for (int s = 0; s < Vec<F>::N; ++s) x[s] = x[s] + r[s];
      }
    const size_t o = (size_t)node * a.B + cw0;
#pragma unroll
    for (int s = 0; s < Vec<F>::N; ++s) {
      if (cw0 + s >= a.B) break;
      if (a.out_dtype == kF32) reinterpret_cast<float*>(a.out)[o + s] = (float)x[s];
      else reinterpret_cast<double*>(a.out)[o + s] = (double)x[s];
    }
  });
}

// ------------------------------------------------------------ fused on-chip decoder
// IBL_FL_CN64: full check tasks (64 nodes) run a body with the constant edge stride (A/B: 0 = off)
#ifndef IBL_FL_CN64
#define IBL_FL_CN64 1
#endif
// For codes whose messages fit in LDS ((E + N) * 16 B <= 160 KiB, e.g. WLAN N=1944: 142.6 KB), one
// workgroup decodes Vec<F>::N codewords (4 fp32 / 2 fp64, one 16-byte slot per edge and per
// variable) through ALL iterations without touching HBM: the flooding schedule of
// decode_OpenCL_min_sum / decode_OpenCL_belief_propagation (min_sum_decoder_irreg.py:221-287,
// bp_decoder_irreg.py:221-286) as barrier-separated phases over one in-place message array:
//   send (kernels_min_and_BP.cl:12-29); for j = 1..L { CN pass (+ syndrome of its inputs, :206-227);
//   VN pass (:76-123) unless j == L }; APP output (:170-204) from the last CN pass.
// Check and variable nodes own their slots (a node reads all its inputs before writing its outputs
// to the same slots), so one array serves both directions. Node bodies are the per-pass kernels'
// (fl_cn_body / fl_vn_body), same operations in the same order: outputs equal the per-pass path's
// bit for bit. Work inside a phase: tasks of up to 64 same-degree nodes, heaviest first, handed to
// waves by LDS tickets; two counters alternate between phases (reset one phase ahead).
// Early stop is batch-global in the reference (stop when the WHOLE batch's syndrome is zero): pass 1
// runs imax-1 iterations and records each CN pass's syndrome in the same flag words as the per-pass
// path; finalize_iters turns them into L; pass 2 (dL set) re-runs the batch to L only if L < imax-1.
// A message slot holds Vec<F>::N codewords (16 bytes); fused tasks work on a slice of NC of them (slice h:
// codewords h*NC .. h*NC+NC-1), read and written as NC*sizeof(F) bytes at byte offset h*NC*sizeof(F).
template <typename F, int NC> struct Slice;
template <> struct Slice<float, 4> { using T = float4; };
template <> struct Slice<float, 2> { using T = float2; };
template <> struct Slice<double, 2> { using T = double2; };

template <typename F, int NC>
__device__ __forceinline__ void slice_load(const void* base, int slot, int h, F (&v)[NC]) {
  const typename Slice<F, NC>::T r =
      reinterpret_cast<const typename Slice<F, NC>::T*>(base)[slot * (Vec<F>::N / NC) + h];
  const F* e = reinterpret_cast<const F*>(&r);
#pragma unroll
  for (int s = 0; s < NC; ++s) v[s] = e[s];
}
template <typename F, int NC>
__device__ __forceinline__ void slice_store(void* base, int slot, int h, const F (&v)[NC]) {
  typename Slice<F, NC>::T r;
  F* e = reinterpret_cast<F*>(&r);
#pragma unroll
  for (int s = 0; s < NC; ++s) e[s] = v[s];
  reinterpret_cast<typename Slice<F, NC>::T*>(base)[slot * (Vec<F>::N / NC) + h] = r;
}

template <int KIND, typename F, int D, int NC, int CNT = 0>
__device__ __forceinline__ void fused_cn_item(void* msg, int first, int cnt_, int lane, int h, F lm,
                                              bool do_par, int valid, bool& unsat) {
  // CNT > 0: a full task (CNT nodes) — the edge stride is a constant, so one address register serves all
  // D loads and stores through their immediate offsets
  const int cnt = CNT > 0 ? CNT : cnt_;
  F m[D][NC];
#pragma unroll
  for (int j = 0; j < D; ++j) slice_load<F, NC>(msg, first + j * cnt + lane, h, m[j]);
  if (do_par) {
#pragma unroll
    for (int s = 0; s < NC; ++s) unsat |= syndrome_bit<F, D>(m, s) && h * NC + s < valid;
  }
  fl_cn_body<KIND, F, D>(m, lm, [&](int w, const F (&o)[NC]) __attribute__((always_inline)) {
    slice_store<F, NC>(msg, first + w * cnt + lane, h, o);
  });
}

// Variable-edge slot indices: staged into LDS as 16-bit values beside the messages (the fused path
// requires the room for them, capi.hip fused_setup), row k of a task at sfirst + 64k: the D loads share
// one address and take their row offsets as immediates.
template <typename F, int D, int NC>
__device__ __forceinline__ void fused_vn_item(void* msg, const void* chL, const uint16_t* vn_slot, int pos,
                                              int sfirst, int lane, int h, F lm) {
  int sl[D];
#pragma unroll
  for (int k = 0; k < D; ++k) sl[k] = vn_slot[sfirst + 64 * k + lane];
  F c[NC], m[D][NC];
  slice_load<F, NC>(chL, pos, h, c);
#pragma unroll
  for (int k = 0; k < D; ++k) slice_load<F, NC>(msg, sl[k], h, m[k]);
  fl_vn_body<F, D>(c, m, lm, [&](int w, const F (&o)[NC]) __attribute__((always_inline)) {
    slice_store<F, NC>(msg, sl[w], h, o);
  });
}

// CMAX / VMAX: largest check / variable degree with a body (WLAN: checks <= 8, variables up to 11 ->
// fl_fused<.., 8, 16>, without the 16-input check bodies' registers)
template <int KIND, typename F, int CMAX, int VMAX>
__global__ __launch_bounds__((fl_fused_block_of<CMAX, KIND, F>())) void fl_fused(FlFusedArgs a) {
  using V = Vec<F>;
  using VT = typename V::T;
  constexpr int N = V::N;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  VT* msg = reinterpret_cast<VT*>(lds);
  VT* chL = msg + a.n_e;
  // tasks take whole slots (slice 0 of N codewords): half slots (2 fp32 codewords per task, twice the
  // tasks) measured 1.29x slower on C3 (WLAN N=1944) — the per-task latency, not the body, dominates
  constexpr int NCs = N, h = 0;
  int* ctr = reinterpret_cast<int*>(chL + a.n_v);
  const int lane = fl_tid() & 63;
  const F lm = (F)a.llr_max;
  int L = a.imax - 1;
  if (a.dL) {
    L = __builtin_amdgcn_readfirstlane(*a.dL);
    if (L >= a.imax - 1) return;   // no early stop happened: pass 1's outputs stand
  }
  if (fl_tid() < 2) ctr[fl_tid()] = 0;
  // variable-edge slot indices, [ctr x 4][n_vs x u16] after the channel slots
  uint16_t* vs = reinterpret_cast<uint16_t*>(ctr + 4);
  for (int i = fl_tid(); i < a.n_vs; i += fl_bdim()) vs[i] = (uint16_t)a.vn_slot[i];
  __syncthreads();
  int ph = 0;
  const int shard = (int)((fl_bid() * (fl_bdim() >> 6) + (fl_tid() >> 6)) & (kShards - 1));
  // one phase: tasks dealt by ticket; the next phase's counter is reset while this one runs
#ifndef IBL_FUSED_TRACE
#define IBL_FUSED_TRACE 0
#endif
  // phase trace of block 0's first group (diagnostic builds): kFlTraceWords per phase (common.h)
  const int wv = fl_tid() >> 6;
  constexpr int TW = kFlTraceWords;
  uint64_t* tr = (IBL_FUSED_TRACE && a.trace && fl_bid() == 0 && lane == 0) ? a.trace : nullptr;
  if (IBL_FUSED_TRACE && tr && wv == 0) tr[0] = __builtin_readcyclecounter();
  // ---- task bodies (one task = up to 64 same-degree nodes, lane i = node i) ----
  // send: every variable's channel slot and its edge slots
  auto send_task = [&](int t, int grp) __attribute__((always_inline)) {
    const int pos = sload(a.vn_task, 4 * t), cnt = sload(a.vn_task, 4 * t + 1);
    const int d = sload(a.vn_task, 4 * t + 2), sf = sload(a.vn_task, 4 * t + 3);
    if (lane < cnt) {
      // channel staged as [group][variable position] (fl_stage_t): a task reads consecutive slots
      const VT c = reinterpret_cast<const VT*>(a.ch)[(size_t)grp * a.n_v + pos + lane];
      chL[pos + lane] = c;
      for (int k = 0; k < d; ++k) msg[vs[sf + 64 * k + lane]] = c;
    }
  };
  auto cn_task = [&](int t, int valid, bool do_par, bool& unsat) __attribute__((always_inline)) {
    const int first = sload(a.cn_task, 4 * t), cnt = sload(a.cn_task, 4 * t + 1), d = sload(a.cn_task, 4 * t + 2);
    // the constant-stride body exists for degrees <= 8 only; full tasks of larger degrees take the general
    // branch below (every lane < cnt = 64)
    if (IBL_FL_CN64 && cnt == 64 && d <= 8) {
      switch (d) {
#define X(D) case D: if constexpr (D <= CMAX && D <= 8) fused_cn_item<KIND, F, D, NCs, 64>(msg, first, cnt, lane, h, lm, do_par, valid, unsat); break;
        FL_DEG_CASES(X)
#undef X
        default: break;
      }
    } else if (lane < cnt) {
      switch (d) {
#define X(D) case D: if constexpr (D <= CMAX) fused_cn_item<KIND, F, D, NCs>(msg, first, cnt, lane, h, lm, do_par, valid, unsat); break;
        FL_DEG_CASES(X)
#undef X
        default: break;
      }
    }
  };
  auto vn_task = [&](int t) __attribute__((always_inline)) {
    const int pos = sload(a.vn_task, 4 * t), cnt = sload(a.vn_task, 4 * t + 1);
    const int d = sload(a.vn_task, 4 * t + 2), sf = sload(a.vn_task, 4 * t + 3);
    if (lane < cnt) {
      switch (d) {
        case 1: fused_vn_item<F, 1, NCs>(msg, chL, vs, pos + lane, sf, lane, h, lm); break;
#define X(D) case D: if constexpr (D <= VMAX) fused_vn_item<F, D, NCs>(msg, chL, vs, pos + lane, sf, lane, h, lm); break;
        FL_DEG_CASES(X)
#undef X
        default: break;
      }
    }
  };
  // APP output: ch + all inputs of the last CN pass in ascending edge order, unclamped
  auto out_task = [&](int t, int cw0, int valid) __attribute__((always_inline)) {
    const int pos = sload(a.vn_task, 4 * t), cnt = sload(a.vn_task, 4 * t + 1);
    const int d = sload(a.vn_task, 4 * t + 2), sf = sload(a.vn_task, 4 * t + 3);
    if (lane < cnt) {
      const int node = a.vn_node[pos + lane];
      F x[N];
      {
        const VT r = chL[pos + lane];
#pragma unroll
        for (int s = 0; s < N; ++s) x[s] = V::get(r, s);
      }
      if (L > 0)
        for (int k = 0; k < d; ++k) {
          const VT r = msg[vs[sf + 64 * k + lane]];
#pragma unroll
          for (int s = 0; s < N; ++s) x[s] = x[s] + V::get(r, s);
        }
      const size_t o = (size_t)node * a.B + cw0;
      if (a.out_dtype == kF32) {
        float* p = reinterpret_cast<float*>(a.out) + o;
        if constexpr (N == 4) {
          if (a.aligned && valid >= 4) {
            *reinterpret_cast<float4*>(p) = make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]);
            return;
          }
        }
#pragma unroll
        for (int s = 0; s < N; ++s)
          if (s < valid) p[s] = (float)x[s];
      } else {
        double* p = reinterpret_cast<double*>(a.out) + o;
        if constexpr (N == 2) {
          if (a.aligned && valid >= 2) {
            *reinterpret_cast<double2*>(p) = make_double2((double)x[0], (double)x[1]);
            return;
          }
        }
#pragma unroll
        for (int s = 0; s < N; ++s)
          if (s < valid) p[s] = (double)x[s];
      }
    }
  };

  // ---- phases separated by barriers
  auto phase = [&](int ntasks, auto&& body) __attribute__((always_inline)) {
    int* c = ctr + (ph & 1);
    if (fl_tid() == 0) ctr[(ph + 1) & 1] = 0;
    int taken = 0;
    for (;;) {
      const int t = take_ticket(c, lane);
      if (t >= ntasks) break;
      if constexpr (IBL_FUSED_TRACE) {
        if (tr && taken == 0) tr[TW * ph + 33 + wv] = __builtin_readcyclecounter();
      }
      body(t);
      if constexpr (IBL_FUSED_TRACE) {
        if (tr && taken == 0) tr[TW * ph + 49 + wv] = __builtin_readcyclecounter();
      }
      ++taken;
    }
    if constexpr (IBL_FUSED_TRACE) {
      if (tr) {
        tr[TW * ph + 1 + wv] = __builtin_readcyclecounter();
        tr[TW * ph + 17 + wv] = (uint64_t)taken;
      }
    }
    __syncthreads();
    ++ph;
    if constexpr (IBL_FUSED_TRACE) {
      if (tr && wv == 0) tr[TW * ph] = __builtin_readcyclecounter();
    }
  };
  for (int grp = fl_bid(); grp < a.ngroups; grp += fl_gdim()) {
    const int cw0 = grp * N;
    const int valid = a.B - cw0;
    phase(a.n_vn_tasks, [&](int t) __attribute__((always_inline)) { send_task(t, grp); });
    for (int j = 1; j <= L; ++j) {
      const bool do_par = a.unsat != nullptr;
      bool unsat = false;
      phase(a.n_cn_tasks, [&](int t) __attribute__((always_inline)) { cn_task(t, valid, do_par, unsat); });
      if (do_par && __ballot(unsat) != 0ull && lane == 0) atomicOr(&a.unsat[(size_t)(j - 1) * kShards + shard], 1);
      if (j == L) break;
      phase(a.n_vn_tasks, [&](int t) __attribute__((always_inline)) { vn_task(t); });
    }
    phase(a.n_vn_tasks, [&](int t) __attribute__((always_inline)) { out_task(t, cw0, valid); });
    tr = nullptr;   // trace the first group only
  }
}

// ---------------------------------------------------------------------- launchers
hipError_t launch_fl_stage(const void* x, int in_dtype, int n, int B, void* dst, int prec, int ldb, int rule,
                           int32_t* bad, hipStream_t s) {
  const size_t total = (size_t)n * ldb;
  const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
  if (prec == kF32)
    hipLaunchKernelGGL(fl_stage<float>, dim3(grid), dim3(256), 0, s, x, in_dtype, n, B, (float*)dst, ldb, rule, bad);
  else
    hipLaunchKernelGGL(fl_stage<double>, dim3(grid), dim3(256), 0, s, x, in_dtype, n, B, (double*)dst, ldb, rule, bad);
  return hipGetLastError();
}

hipError_t launch_fl_stage_t(const void* x, int in_dtype, int n, int B, const int32_t* perm, void* dst, int prec,
                             int rule, int32_t* bad, hipStream_t s) {
  const int cwl = prec == kF32 ? 4 : 2;
  const size_t tiles = (size_t)((n + 63) / 64) * (size_t)((((B + cwl - 1) / cwl) + 31) / 32);
  const int grid = (int)std::max<size_t>(1, std::min<size_t>(tiles, 8192));
  if (prec == kF32)
    hipLaunchKernelGGL(fl_stage_t<float>, dim3(grid), dim3(256), 0, s, x, in_dtype, n, B, perm, (float4*)dst, rule, bad);
  else
    hipLaunchKernelGGL(fl_stage_t<double>, dim3(grid), dim3(256), 0, s, x, in_dtype, n, B, perm, (double2*)dst, rule, bad);
  return hipGetLastError();
}

// Host-side operand checks before a launch: a missing array would fault the device, not fail the call.
static bool fl_args_ok(const FlArgs& a, int which) {
  if (!a.out || !a.start || !a.deg || !a.tgt || a.ldb <= 0 || a.n_nodes < 0 || a.B <= 0 || a.B > a.ldb) return false;
  if (which == 0) return a.in && (a.fold_mode == 0 || (a.fold && a.fout && a.ch));   // check pass
  if (which == 1) return a.in && a.ch;                                              // variable pass
  return a.ch != nullptr;                                                           // send
}

hipError_t launch_fl_send(const FlArgs& a, int prec, hipStream_t s) {
  if (!fl_args_ok(a, 2)) return hipErrorInvalidValue;
  const size_t total = (size_t)a.n_nodes * (a.ldb / 4);
  const int grid = (int)std::min<size_t>((total + 255) / 256, 8192);
  if (prec == kF32) hipLaunchKernelGGL(fl_send<float>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(fl_send<double>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

static const void* fl_kernel(int which, int kind, int prec, int maxd) {
  const bool f32 = prec == kF32, small = maxd <= 8;
  if (which == 0) {
    if (kind == 0)
      return f32 ? (small ? (const void*)fl_cn<0, float, 8> : (const void*)fl_cn<0, float, 16>)
                 : (small ? (const void*)fl_cn<0, double, 8> : (const void*)fl_cn<0, double, 16>);
    return f32 ? (small ? (const void*)fl_cn<1, float, 8> : (const void*)fl_cn<1, float, 16>)
               : (small ? (const void*)fl_cn<1, double, 8> : (const void*)fl_cn<1, double, 16>);
  }
  return f32 ? (small ? (const void*)fl_vn<float, 8> : (const void*)fl_vn<float, 16>)
             : (small ? (const void*)fl_vn<double, 8> : (const void*)fl_vn<double, 16>);
}

int fl_block(int which, int kind, int prec, int maxd) {
  if (which == 0 && kind == 1 && (maxd > 8 || prec == kF64)) return fl_block_of<0, 16, 1, float>();
  if (which == 0 && kind == 0 && maxd > 8 && prec == kF32) return fl_block_of<0, 16, 0, float>();
  return fl_block_of<1, 8>();
}

hipError_t launch_fl_cn(const FlArgs& a, int kind, int prec, int maxd, int grid, hipStream_t s) {
  if (!fl_args_ok(a, 0)) return hipErrorInvalidValue;
  FlArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_kernel(0, kind, prec, maxd), dim3(grid), dim3(fl_block(0, kind, prec, maxd)), p, 0, s);
}

hipError_t launch_fl_vn(const FlArgs& a, int prec, int maxd, int grid, hipStream_t s) {
  if (!fl_args_ok(a, 1)) return hipErrorInvalidValue;
  FlArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_kernel(1, 0, prec, maxd), dim3(grid), dim3(fl_block(1, 0, prec, maxd)), p, 0, s);
}

template <int KIND, typename F>
static const void* fl_fused_kernel_t(int cmax, int vmax) {
  if (cmax <= 8) return vmax <= 8 ? (const void*)fl_fused<KIND, F, 8, 8> : (const void*)fl_fused<KIND, F, 8, 16>;
  return (const void*)fl_fused<KIND, F, 16, 16>;
}
static const void* fl_fused_kernel(int kind, int prec, int cmax, int vmax) {
  if (kind == 0) return prec == kF32 ? fl_fused_kernel_t<0, float>(cmax, vmax) : fl_fused_kernel_t<0, double>(cmax, vmax);
  return prec == kF32 ? fl_fused_kernel_t<1, float>(cmax, vmax) : fl_fused_kernel_t<1, double>(cmax, vmax);
}

hipError_t fl_fused_occupancy(int kind, int prec, int cmax, int vmax, size_t lds, int* blocks_per_cu, int* block) {
  const void* f = fl_fused_kernel(kind, prec, cmax, vmax);
  *block = fl_fused_block(kind, prec, cmax);
  hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (e != hipSuccess) return e;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, *block, lds);
}

hipError_t launch_fl_fused(const FlFusedArgs& a, int kind, int prec, int cmax, int vmax, int grid, size_t lds,
                           hipStream_t s) {
  FlFusedArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_fused_kernel(kind, prec, cmax, vmax), dim3(grid),
                         dim3(fl_fused_block(kind, prec, cmax)), p, lds, s);
}

static bool fl_small_ok(const FlArgs& a, bool vn) {
  return a.info && a.task && a.in && a.out && a.tgt && (!vn || a.ch) && a.nwords >= 1 && a.ldb > 0 && a.B > 0;
}
template <int KIND>
static const void* fl_cn_small_kernel(int prec, int maxd) {
  if (prec == kF32) return maxd <= 8 ? (const void*)fl_cn_small<KIND, float, 8> : (const void*)fl_cn_small<KIND, float, 16>;
  return maxd <= 8 ? (const void*)fl_cn_small<KIND, double, 8> : (const void*)fl_cn_small<KIND, double, 16>;
}
static const void* fl_small_kernel(int which, int kind, int prec, int maxd) {
  if (which == 0) return kind == 0 ? fl_cn_small_kernel<0>(prec, maxd) : fl_cn_small_kernel<1>(prec, maxd);
  if (which == 1)
    return prec == kF32 ? (maxd <= 8 ? (const void*)fl_vn_small<float, 8> : (const void*)fl_vn_small<float, 16>)
                        : (maxd <= 8 ? (const void*)fl_vn_small<double, 8> : (const void*)fl_vn_small<double, 16>);
  return prec == kF32 ? (const void*)fl_dec_small<float> : (const void*)fl_dec_small<double>;
}
hipError_t launch_fl_cn_small(const FlArgs& a, int kind, int prec, int maxd, int grid, hipStream_t s) {
  if (!fl_small_ok(a, false)) return hipErrorInvalidValue;
  FlArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_small_kernel(0, kind, prec, maxd), dim3(grid), dim3(kFlSmallBlock), p, 0, s);
}
hipError_t launch_fl_vn_small(const FlArgs& a, int prec, int maxd, int grid, hipStream_t s) {
  if (!fl_small_ok(a, true)) return hipErrorInvalidValue;
  FlArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_small_kernel(1, 0, prec, maxd), dim3(grid), dim3(kFlSmallBlock), p, 0, s);
}
hipError_t launch_fl_dec_small(const FlDecArgs& a, int prec, int grid, hipStream_t s) {
  if (!a.info || !a.task || !a.vin0 || !a.vin1 || !a.ch || !a.out || a.nwords < 1) return hipErrorInvalidValue;
  FlDecArgs args = a;
  void* p[] = {&args};
  return hipLaunchKernel(fl_small_kernel(2, 0, prec, 0), dim3(grid), dim3(kFlSmallBlock), p, 0, s);
}
hipError_t fl_small_private_bytes(int kind, int prec, int cn_maxd, int vn_maxd, size_t* bytes, const char** name) {
  const struct { const void* f; const char* n; } ks[] = {{fl_small_kernel(0, kind, prec, cn_maxd), "fl_cn_small"},
                                                           {fl_small_kernel(1, kind, prec, vn_maxd), "fl_vn_small"},
                                                           {fl_small_kernel(2, kind, prec, 0), "fl_dec_small"}};
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

hipError_t launch_fl_dec(const FlDecArgs& a, int prec, int grid, hipStream_t s) {
  if (prec == kF32) hipLaunchKernelGGL(fl_dec<float>, dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(fl_dec<double>, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t fl_private_bytes(int kind, int prec, int cn_maxd, int vn_maxd, bool fused, size_t* bytes,
                            const char** name) {
  const struct { const void* f; const char* n; } ks[] = {
      {fl_kernel(0, kind, prec, cn_maxd), "fl_cn"}, {fl_kernel(1, kind, prec, vn_maxd), "fl_vn"},
      {fused ? fl_fused_kernel(kind, prec, cn_maxd, vn_maxd) : nullptr, "fl_fused"}};
  *bytes = 0;
  *name = "";
  for (const auto& k : ks) {
    if (!k.f) continue;
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

hipError_t fl_occupancy(int which, int kind, int prec, int maxd, int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fl_kernel(which, kind, prec, maxd),
                                                      fl_block(which, kind, prec, maxd), 0);
}

}  // namespace ibl
