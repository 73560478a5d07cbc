// LDS-DMA operand loaders and fragment readers of the g4 engine (gemm_g4.hip), shared with the
// halo-tile direct convolution (conv_halo.hip). Layouts: see the header comment of gemm_g4.hip.
#pragma once
#include "common.h"
#include "gemm_params.h"

namespace tfk {
namespace g4 {

constexpr int BK = 64;
constexpr unsigned OOB = 0x80000000u;
constexpr int NREC = 0x7FFFFFF0;

enum { KIN = 0, KOUT = 1, CONV_FWD = 2, CONV_WGRAD = 3 };

__device__ __forceinline__ unsigned fdiv(unsigned x, unsigned mul, int shift) { return (__umulhi(x, mul) + x) >> shift; }

__device__ __forceinline__ int swz64(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

typedef int i32x8 __attribute__((ext_vector_type(8)));

// Two 16-B fragment halves -> the 32-B operand of one scaled fp8 MFMA (16x16x128).
__device__ __forceinline__ i32x8 pack8(bf16x8 lo, bf16x8 hi) {
  const u32x4 a = __builtin_bit_cast(u32x4, lo), b = __builtin_bit_cast(u32x4, hi);
  i32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// Fragment (16 image rows from rb, K-half kk) of an operand image with ROWS rows.
template <bool KO>
__device__ __forceinline__ bf16x8 frag(const char* img, int rb, int kk) {
  const int l = threadIdx.x & 63;
  if constexpr (!KO) {
    const int row = rb + (l & 15);
    const int c = kk * 4 + (l >> 4);
    return *(const bf16x8*)(img + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  } else {
    const char* b = img + (rb >> 6) * 8192;
    const int g = l >> 4, i = l & 15, q = i >> 2, pc = i & 3;
    const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
    const int ch = ((rb & 63) >> 3) + (pc >> 1);
    const int o0 = k0 * 128 + ((ch ^ swz64(k0)) << 4) + (pc & 1) * 8;
    const int o1 = k1 * 128 + ((ch ^ swz64(k1)) << 4) + (pc & 1) * 8;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(b + o0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LDS_AS bf16x4*)(b + o1));
    bf16x8 r;
    r.lo = lo;
    r.hi = hi;
    return r;
  }
}

// Per-thread DMA plan of one operand: ROWS/32 instructions per K-tile. Instruction j (of ROWS/8,
// wave w takes j = 4i + w) fills image bytes [j*1024, j*1024+1024).
// SMALLC: also compile the Cin < 64 conv-forward gather (off in the 128-VGPR single-stage kernels,
// which the host never gives such a conv)
template <int ROWS, int MODE, int NW, bool SMALLC = true>
struct Loader {
  static constexpr int NI = ROWS / 8 / NW;  // DMA instructions per thread per K-tile
  // dense: byte offset from the tile origin at K-tile 0; conv: image index n of the lane's pixel
  unsigned off[NI];
  // conv gather: input-space origin (p*sh - ph, q*sw - pw) of the lane's output pixel
  int ch[NI], cw[NI];

  // row (K-inner) / column (K-outer) of instruction i's lane inside the tile, and its k in a K-tile
  __device__ __forceinline__ static int row_of(int i, int w, int lane) {
    const int j = NW * i + w;
    if constexpr (MODE == KOUT || MODE == CONV_WGRAD) return (j >> 3) * 64 + 8 * ((lane & 7) ^ swz64((j & 7) * 8 + (lane >> 3)));
    else return 8 * j + (lane >> 3);
  }
  __device__ __forceinline__ static int k_of(int i, int w, int lane) {
    const int j = NW * i + w;
    if constexpr (MODE == KOUT || MODE == CONV_WGRAD) return (j & 7) * 8 + (lane >> 3);
    else return 8 * ((lane & 7) ^ (((8 * j + (lane >> 3)) >> 1) & 7));
  }

  __device__ __forceinline__ void init(const GemmParams& p, int lane, int w, long long ld, int row0, int rows) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = row_of(i, w, lane), kl = k_of(i, w, lane);
      if constexpr (MODE == KIN) {
        off[i] = (unsigned)(((long long)r * ld + kl) * 2);
      } else if constexpr (MODE == KOUT) {
        off[i] = (unsigned)(((long long)kl * ld + r) * 2);
      } else if constexpr (MODE == CONV_WGRAD) {
        // column (r, s, c) of the im2col operand is fixed for the kernel: keep the tap's input
        // offset and the channel; columns past N are flagged invalid (top bit of off)
        const int col = row0 + r;
        const int cc = min(col, rows - 1);
        const int rs = cc / p.Cin, c = cc - rs * p.Cin, rr = rs / p.S, ss = rs - rr * p.S;
        ch[i] = rr * p.dh - p.ph;
        cw[i] = ss * p.dw - p.pw;
        off[i] = (unsigned)c | (col < rows ? 0u : OOB);
      } else {
        const int m = min(row0 + r, rows - 1);
        const int PQ = p.P * p.Q;
        const int n = m / PQ, rem = m - n * PQ, pp = rem / p.Q, qq = rem - pp * p.Q;
        ch[i] = pp * p.sh - p.ph;
        cw[i] = qq * p.sw - p.pw;
        // input pixel index of tap (0, 0) (may be negative in the padding: only used when in range;
        // x < 2^30 elements, checked by tfk_g4_ok, so 32-bit pixel / element math suffices); for
        // Cin >= 64 premultiplied by Cin (element index), so a K-tile's address needs no multiply
        const int pix0 = (n * p.H + ch[i]) * p.W + cw[i];
        off[i] = (unsigned)(SMALLC && p.Cin < BK ? pix0 : pix0 * p.Cin);
      }
    }
  }

  // Issue this thread's DMA instructions of K-tile kt into image `img`. base = tile origin;
  // lim = rows left from the tile origin. Interior tiles with a full K-tile skip every edge test.
  // en = false: every lane's offset is out of range -> the DMA writes zeros and touches no memory
  // (lets a pipelined loop issue unconditionally, keeping its MFMA / DMA region one basic block)
  __device__ __forceinline__ void issue(const GemmParams& p, const char* base, long long step, int kt, int lim,
                                        char* img, int w, int lane, bool en = true, int only = -1) const {
    const int krem = p.K - kt * BK;
    const bool inner = lim >= ROWS && krem >= BK;  // block-uniform
    if constexpr (MODE == CONV_WGRAD) {
      __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, NREC, 0x00020000);
      const unsigned PQ = (unsigned)(p.P * p.Q);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (only >= 0 && i != only) continue;
        const unsigned pix = (unsigned)(kt * BK + k_of(i, w, lane));
        const unsigned n = fdiv(pix, p.fd_pq_mul, p.fd_pq_shift), rem = pix - n * PQ;
        const unsigned pp = fdiv(rem, p.fd_q_mul, p.fd_q_shift), qq = rem - pp * (unsigned)p.Q;
        const int h = (int)pp * p.sh + ch[i], wq = (int)qq * p.sw + cw[i];
        const bool ok = !(off[i] & OOB) && (int)pix < p.K && (unsigned)h < (unsigned)p.H && (unsigned)wq < (unsigned)p.W;
        const unsigned vo = ok && en ? (unsigned)(((((long long)n * p.H + h) * p.W + wq) * p.Cin + off[i]) * 2) : OOB;
        lds_dma<16>(rsrc, (LDS_AS void*)(img + (NW * i + w) * 1024), vo);
      }
    } else if constexpr (MODE == CONV_FWD) {
      __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, NREC, 0x00020000);
      if (!SMALLC || p.Cin >= BK) {
        // K-tile kt covers tap (r, s) = divmod(kt*64 / Cin, S) and channels c0..c0+63 (Cin % 64 == 0);
        // the tap's element shift and channel offset are block-uniform (scalar), per lane: adds and
        // the bounds test (off[] holds the premultiplied element index of tap (0, 0))
        const int k0 = kt * BK, rs = k0 / p.Cin, c0 = k0 - rs * p.Cin;
        const int r = rs / p.S, s = rs - r * p.S;
        const int rdh = r * p.dh, sdw = s * p.dw, tapc = (rdh * p.W + sdw) * p.Cin + c0;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if (only >= 0 && i != only) continue;
          const int h = ch[i] + rdh, wq = cw[i] + sdw;
          const bool ok = (inner || row_of(i, w, lane) < lim) && (unsigned)h < (unsigned)p.H && (unsigned)wq < (unsigned)p.W;
          const unsigned vo = ok && en ? (off[i] + (unsigned)(tapc + k_of(i, w, lane))) * 2u : OOB;
          lds_dma<16>(rsrc, (LDS_AS void*)(img + (NW * i + w) * 1024), vo);
        }
      } else {
        // Cin % 8 == 0, Cin < 64 (the stem's 3 channels padded to 8): a K-tile spans 64/Cin taps and
        // each lane's 16-B chunk is 8 channels of ONE tap -- per-lane (tap, c) by magic-number
        // division (host: fd_pq = Cin, fd_q = S); k >= K (the ragged last K-tile) reads zeros
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if (only >= 0 && i != only) continue;
          const unsigned k = (unsigned)(kt * BK + k_of(i, w, lane));
          const unsigned rs = fdiv(k, p.fd_pq_mul, p.fd_pq_shift), c = k - rs * (unsigned)p.Cin;
          const unsigned r = fdiv(rs, p.fd_q_mul, p.fd_q_shift), sx = rs - r * (unsigned)p.S;
          const int h = ch[i] + (int)r * p.dh, wq = cw[i] + (int)sx * p.dw;
          const bool ok = (int)k < p.K && (inner || row_of(i, w, lane) < lim) && (unsigned)h < (unsigned)p.H &&
                          (unsigned)wq < (unsigned)p.W;
          const int pix = (int)off[i] + (int)r * p.dh * p.W + (int)sx * p.dw;
          const unsigned vo = ok && en ? (unsigned)(pix * p.Cin + (int)c) * 2u : OOB;
          lds_dma<16>(rsrc, (LDS_AS void*)(img + (NW * i + w) * 1024), vo);
        }
      }
    } else {
      __amdgpu_buffer_rsrc_t rsrc =
          __builtin_amdgcn_make_buffer_rsrc((void*)(base + kt * step), (short)0, NREC, 0x00020000);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if (only >= 0 && i != only) continue;
        unsigned vo = off[i];
        if (!inner) vo = (row_of(i, w, lane) < lim && k_of(i, w, lane) < krem) ? vo : OOB;
        if (!en) vo = OOB;
        lds_dma<16>(rsrc, (LDS_AS void*)(img + (NW * i + w) * 1024), vo);
      }
    }
  }
};

}  // namespace g4
}  // namespace tfk
