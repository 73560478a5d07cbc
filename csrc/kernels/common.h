// Common device helpers for the tfk gfx950 (CDNA4) kernel library.
// Everything here is written for wave64 / MFMA / 160 KiB LDS; no CUDA shims.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define LDS_AS __attribute__((address_space(3)))
#define TFK_WAVE 64

// LDS-DMA (buffer_load ... lds) of BYTES (16 or 4) per lane into LDS at `lds` + 16*lane (4*lane),
// issued from inline asm: hipcc 7.2's waitcnt pass does not see it. Through the builtin it treats
// every later ds_read_b64_tr_b16 as possibly reading the DMA's bytes and puts s_waitcnt vmcnt(0) in
// front of it, so a transposed read of stage s waited for stage s^1's just-issued DMA (the K-outer
// GEMMs and the weight-gradient kernels lost their DMA / MFMA overlap; plain ds_read_b128 is not
// affected). Every caller waits for its DMAs itself (s_waitcnt vmcnt + barrier) before reading a
// stage or reusing the LDS; M0 is written only here (no builtin LDS-DMA remains in the library, so
// no compiler-tracked M0 value is clobbered).
template <int BYTES>
__device__ __forceinline__ void lds_dma(__amdgpu_buffer_rsrc_t rsrc, LDS_AS void* lds, unsigned voff) {
  static_assert(BYTES == 16 || BYTES == 4, "dwordx4 or dword");
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)lds);
  if constexpr (BYTES == 16)
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rsrc) : "memory");
  else
    asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m0), "v"(voff), "s"(rsrc) : "memory");
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)

// Wave-wide reductions without the LDS: DPP within each 16-lane row (quad_perm xor 1, xor 2, then
// half-row mirror and row mirror -- every lane of a group already holds the group's value, so any
// cross-group pairing completes the butterfly) and gfx950's v_permlane16/32_swap across rows.
// (__shfl_xor is a ds_bpermute plus an lgkmcnt(0) wait per step: 6 LDS round trips per reduction.)
// Every lane ends with the bitwise-same value (each step adds the same two operands on both sides).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float lane_swap16(float v, float& other) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  other = __uint_as_float(a[1]);
  return __uint_as_float(a[0]);
}
__device__ __forceinline__ float lane_swap32(float v, float& other) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  other = __uint_as_float(a[1]);
  return __uint_as_float(a[0]);
}
// sum over the lane pair (l, l ^ O), O in {8, 16, 32}: row_ror 8 within a 16-lane row, or a
// permlane swap across rows (both lanes get the same operands in the same order)
template <int O>
__device__ __forceinline__ float xor_sum(float v) {
  static_assert(O == 8 || O == 16 || O == 32, "xor_sum: O in {8, 16, 32}");
  if constexpr (O == 8) {
    return v + dpp_f<0x128>(v);
  } else {
    float o;
    const float a = O == 16 ? lane_swap16(v, o) : lane_swap32(v, o);
    return a + o;
  }
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  float o;
  float a = lane_swap16(v, o);
  v = a + o;
  a = lane_swap32(v, o);
  return a + o;
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  float o;
  float a = lane_swap16(v, o);
  v = fmaxf(a, o);
  a = lane_swap32(v, o);
  return fmaxf(a, o);
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

// tanh from the native exp (v_exp_f32) and reciprocal (v_rcp_f32): 1 - 2/(1 + e^{2u}), saturating to
// +-1 through e^{2u} = inf / 0. Absolute error ~1e-7 (the libm tanhf is ~10x the VALU work, which made
// BERT's GELU-backward dgrad epilogue VALU-bound: 133 us vs 59 us for the plain dgrad). __fdividef
// still lowered to the IEEE division sequence here (v_div_scale / div_fmas / div_fixup per call).
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u));
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}

// Activation codes shared by GEMM epilogues and elementwise kernels: 0 none, 1 relu, 2 gelu(tanh), 3 tanh.
__device__ __forceinline__ float act_apply(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : (act == 2 ? gelu_tanh(v) : (act == 3 ? fast_tanh(v) : v));
}
// derivative at the PRE-activation z
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 1) return z > 0.f ? 1.f : 0.f;
  if (act == 2) return gelu_tanh_grad(z);
  if (act == 3) { const float t = fast_tanh(z); return 1.f - t * t; }
  return 1.f;
}

// 8-element forms with the (wave-uniform) activation switch taken once per chunk instead of once per
// element: the per-element switch compiled to a chain of scalar compares and branches per element.
__device__ __forceinline__ void act_apply8(float (&f)[8], int act) {
  if (act == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = gelu_tanh(f[e]);
  } else if (act == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaxf(f[e], 0.f);
  } else if (act == 3) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fast_tanh(f[e]);
  }
}
// f[e] *= act'(z[e])
__device__ __forceinline__ void act_grad_mul8(float (&f)[8], const bf16x8& z, int act) {
  if (act == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= gelu_tanh_grad(bf2f(z[e]));
  } else if (act == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] *= bf2f(z[e]) > 0.f ? 1.f : 0.f;
  } else if (act == 3) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = fast_tanh(bf2f(z[e]));
      f[e] *= 1.f - t * t;
    }
  }
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 'XCD swizzle must be bijective'):
// blocks b and b+8 share an XCD under round-robin dispatch, so give each XCD a contiguous range
// of logical tile ids -> neighbouring tiles (sharing an A panel) hit the same 4 MiB L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, loc = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Counter-based RNG (Philox-lite, 2 rounds of mulhi mixing) for dropout / synthetic data.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t x = idx * 0x9E3779B97F4A7C15ull ^ (seed + 0xD1B54A32D192ED03ull);
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float u01(uint32_t h) { return (h >> 8) * (1.0f / 16777216.0f); }

// Dropout seeds = host per-site salt + a per-step device key. The key (a model's rng state
// [counter, key], advanced on the device at the start of every training step by rng_advance) makes
// masks change per step INSIDE a replayed hipGraph; the salt separates the sites of one step. The
// launchers pick up the key pointer registered by tfk_set_seed_key (null: salt only).
__device__ __forceinline__ unsigned long long eff_seed(unsigned long long salt, const unsigned long long* key) {
  return key ? salt + *key : salt;
}
extern "C" const unsigned long long* tfk_seed_key();
// 32-bit integer hash ("lowbias32": 2 multiplies, 3 xor-shifts, all 32-bit) for the per-element
// attention-dropout masks, which are regenerated in every attention pass: the 64-bit hash_u32
// above costs ~35 VALU ops per element there and was the largest cost of the dropout passes.
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// Elementwise dropout masks (GEMM epilogues, dropout kernels, LayerNorm-backward dropout): the
// 64-bit seed (salt + per-step key) folds once into a 32-bit stream seed; ONE hash32 per group of 4
// consecutive elements gives 4 mask bytes -- element i is kept iff byte (i & 3) of
// hash32(s32 ^ (i >> 2)) >= thr = round(256 p), scaled by 256 / (256 - thr) (exactly unbiased).
// The effective drop rate is thr / 256 (p = 0.1 -> 0.1016); rates 0 < p < 1/512 and p > 255.5/256
// are not representable and are rejected by the Python layer (ops/elementwise.py check_rate).
// A hash per element (two quarter-rate multiplies + shifts) was the largest VALU cost of the
// dropout-carrying GEMM epilogues (ops/elementwise.py dropout_keep is the bit-exact CPU copy).
__device__ __forceinline__ uint32_t drop_seed32(unsigned long long s) {
  return hash32((uint32_t)s ^ hash32((uint32_t)(s >> 32) ^ 0x9E3779B9u));
}
__host__ __device__ __forceinline__ int drop_thr8(float p) {
  const int t = (int)(p * 256.f + 0.5f);
  return t > 255 ? 255 : (t < 0 ? 0 : t);
}
__host__ __device__ __forceinline__ float drop_scale8(float p) { return 256.f / (float)(256 - drop_thr8(p)); }
__device__ __forceinline__ bool drop_keep1(uint32_t s32, unsigned long long idx, int thr) {
  return ((hash32(s32 ^ (uint32_t)(idx >> 2)) >> (8 * (unsigned)(idx & 3))) & 0xffu) >= (uint32_t)thr;
}
// keep bits (bit e) of elements base .. base+7, any base (two hashes when base % 4 == 0)
__device__ __forceinline__ unsigned drop_keep8(uint32_t s32, unsigned long long base, int thr) {
  unsigned m = 0;
  if ((base & 3) == 0) {
    const uint32_t h0 = hash32(s32 ^ (uint32_t)(base >> 2)), h1 = hash32(s32 ^ (uint32_t)((base >> 2) + 1));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      m |= ((h0 >> (8 * e)) & 0xffu) >= (uint32_t)thr ? (1u << e) : 0u;
      m |= ((h1 >> (8 * e)) & 0xffu) >= (uint32_t)thr ? (1u << (e + 4)) : 0u;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) m |= drop_keep1(s32, base + e, thr) ? (1u << e) : 0u;
  }
  return m;
}
