// MX (OCP e4m3 + e8m0) block quantization helpers shared by the standalone quantizers (fp8.hip)
// and the GEMM epilogue that emits MX operands directly (gemm_epilogue.h, EPI_BF16_EXT_MX).
#pragma once
#include "common.h"

namespace tfk {
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// scale exponent e = ceil(log2(amax / 448)) from the bf16 bit pattern of amax (-127: all-zero block)
__device__ __forceinline__ int mx_exp_from_bits(unsigned amax_bits) {
  const float amax = __uint_as_float(amax_bits << 16);
  int ex = amax > 0.f ? (int)ceilf(log2f(amax * (1.f / 448.f))) : -127;
  return ex < -127 ? -127 : (ex > 127 ? 127 : ex);
}

// 16 packed bf16 pairs (K order) -> 8 words of e4m3 bytes; returns the exponent
__device__ __forceinline__ int mx_block_pk(const unsigned (&p)[16], unsigned (&w)[8]) {
  u16x2 m = {0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const unsigned a = p[i] & 0x7fff7fffu;
    m = __builtin_elementwise_max(m, *(const u16x2*)&a);
  }
  const int ex = mx_exp_from_bits(m[0] > m[1] ? m[0] : m[1]);
  const float s = ldexpf(1.f, ex < -126 ? -126 : ex);  // all-zero block: any normal scale gives 0
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s16x2 r = {0, 0};
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, *(const bf16x2*)&p[2 * k], s, false);
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, *(const bf16x2*)&p[2 * k + 1], s, true);
    w[k] = *(const unsigned*)&r;
  }
  return ex;
}

}  // namespace tfk
