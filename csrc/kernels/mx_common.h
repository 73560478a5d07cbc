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

// Both MX quantizations of a [32 rows][W] bf16 tile in LDS (row stride ld elements) whose rows are
// global rows r0 .. r0+31 of an [M][W] tensor: row blocks -> qr [M][W] / sr [M][W/32], column
// pairs (one 32-bit LDS word per row holds both columns) -> qc [W][M] / sc [W][M/32]. Every thread
// of the block participates (NT threads); W % 32 == 0, M % 32 == 0, r0 % 32 == 0.
template <int NT>
__device__ __forceinline__ void mx_rows32_out(const bf16* tile, int ld, int W, long long M, int r0, unsigned char* qr,
                                              unsigned char* sr, unsigned char* qc, unsigned char* sc) {
  const int NB = W / 32;
  for (int k = threadIdx.x; k < 32 * NB; k += NT) {
    const int lr = k / NB, blk = k - lr * NB;
    unsigned pp[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const u32x4 h = *(const u32x4*)(tile + lr * ld + blk * 32 + q4 * 8);
      pp[4 * q4] = h[0]; pp[4 * q4 + 1] = h[1]; pp[4 * q4 + 2] = h[2]; pp[4 * q4 + 3] = h[3];
    }
    unsigned w[8];
    const int ex = mx_block_pk(pp, w);
    unsigned char* dst = qr + (long long)(r0 + lr) * W + blk * 32;
    *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
    *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
    sr[(long long)(r0 + lr) * NB + blk] = (unsigned char)(ex + 127);
  }
  for (int cp = threadIdx.x; cp < W / 2; cp += NT) {
    const int col = 2 * cp;
    unsigned lo[16], hi[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const unsigned a = *(const unsigned*)(tile + (2 * r) * ld + col);
      const unsigned b = *(const unsigned*)(tile + (2 * r + 1) * ld + col);
      lo[r] = __builtin_amdgcn_perm(b, a, 0x05040100u);
      hi[r] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    }
    unsigned w[8];
    int ex = mx_block_pk(lo, w);
    unsigned char* dst = qc + (long long)col * M + r0;
    *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
    *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
    sc[(long long)col * (M / 32) + r0 / 32] = (unsigned char)(ex + 127);
    ex = mx_block_pk(hi, w);
    dst += M;
    *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
    *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
    sc[(long long)(col + 1) * (M / 32) + r0 / 32] = (unsigned char)(ex + 127);
  }
}

}  // namespace tfk
