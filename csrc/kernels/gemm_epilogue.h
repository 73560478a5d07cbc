// Shared epilogue of the tfk MFMA GEMM kernels (gemm.hip bf16 engine, fp8.hip MX-fp8 engine).
// Accumulator layout: acc[i][j] of lane l holds C[m][n..n+3] for the wave tile (TM x TN) at
// (wm*TM, wn*TN) of the block tile, m = i*16 + (l&15), n = j*16 + (l>>4)*4.
#pragma once
#include "common.h"
#include "gemm_params.h"
#include "mx_common.h"

#include <type_traits>

namespace tfk {

// BNR: + fused BN-backward reduction; EXT: + aux (pre-activation) store, activation-backward
// multiplier and dropout. Separate instantiations keep the common epilogue small enough to unroll
// fully (a rolled epilogue indexes the accumulators dynamically -> they go to scratch).
// EXT_MX: EXT + MX-fp8 row and column block copies of the output (GemmParams mx_*), quantized from
// the LDS C tile after the store pass (the MX-fp8 engine's producer GEMMs: no separate quantize pass).
// EPI_BF16 ignores p.act: the launcher (gemm.hip tfk_gemm_launch) sends an activated bf16 output to
// EPI_BF16_ACT, whose accumulator pass applies the activation per element. Without it, the runtime
// activation switch compiled to a chain of scalar compares and branches per element in every bf16
// epilogue -- 0.73 ms of a ResNet-50 step, whose convs feed BatchNorms (act = none).
enum EpiMode { EPI_BF16 = 0, EPI_F32 = 1, EPI_BF16_BNR = 2, EPI_BF16_EXT = 3, EPI_BF16_EXT_MX = 4, EPI_BF16_ACT = 5 };

// LDS C-tile swizzle. The accumulator pass stores 8-B pieces (ds_write_b64: 4 groups of 16
// contiguous lanes = 16 rows x one 4-column piece; bank = dword mod 32). With the padded row stride
// (BN + 8 elements = 4 mod 32 dwords for BN = 64/128/256) rows r and r+8 of a group hit the same two
// banks: every accumulator store was a 2-way conflict (the 57-66 % LDS-conflict share of the
// short-K GEMMs, profiles/pmc_resnet50_r5.txt). Swapping the two 8-B halves of each 16-B chunk in
// rows with bit 3 set puts rows 8..15 on the banks rows 0..7 leave free, while 16-B chunks stay
// 16-B aligned for the store pass's ds_read_b128 (which swaps the halves back in registers).
__device__ __forceinline__ int cswz(int row) { return ((row >> 3) & 1) << 2; }  // element XOR of column
__device__ __forceinline__ u32x4 cswap(u32x4 v, int row) {
  return (row & 8) ? u32x4{v[2], v[3], v[0], v[1]} : v;
}
__device__ __forceinline__ bf16x8 crd8(const bf16* p, int row) {  // logical 8-column chunk at its 16-B slot
  return __builtin_bit_cast(bf16x8, cswap(*(const u32x4*)p, row));
}
__device__ __forceinline__ void cwr8(bf16* p, bf16x8 v, int row) {
  *(u32x4*)p = cswap(__builtin_bit_cast(u32x4, v), row);
}

// Both MX quantizations of the final [rows < BM][cols < BN] bf16 tile in LDS (row stride LDS_S):
// row blocks of 32 columns -> mx_qr/mx_sr, column pairs of 32-row blocks (one 32-bit LDS word per
// row holds both columns) -> mx_qc/mx_sc. Same bytes as fp8.hip's mx_quant_dual_kernel.
// Column pass lane map: each 16-lane group is one 32-row group and 16 column pairs, a wave 4 row
// groups -- so the 4 consecutive row groups of a column (4 x 32 B of qc = a full 128-B line, 4 scale
// bytes of sc) go out from one store instruction, while each 32-lane half reads 2 row groups x 16
// column pairs (2-way bank conflict). Lanes walking columns with one row group per wave wrote 32-B
// pieces and single scale bytes 8 KiB apart: 31 us of a 93 us FFN1 forward (profiles/perf_log_r5.md).
template <int BM, int BN, int NT>
__device__ __forceinline__ void mx_tile_out(const GemmParams& p, const bf16* Cs, int lds_s, int m0, int n0) {
  const int tid = threadIdx.x;
  const int rows = min(BM, p.M - m0), cols = min(BN, p.N - n0);
  const long long M = p.M, N = p.N;
  unsigned char* qr = (unsigned char*)p.mx_qr;
  unsigned char* sr = (unsigned char*)p.mx_sr;
  unsigned char* qc = (unsigned char*)p.mx_qc;
  unsigned char* sc = (unsigned char*)p.mx_sc;
  constexpr int NB = BN / 32, RBLK = BM * NB;
#pragma unroll
  for (int k0 = 0; k0 < RBLK; k0 += NT) {
    const int k = k0 + tid, row = k / NB, blk = k - row * NB;
    if (k < RBLK && row < rows && blk * 32 < cols) {
      unsigned pp[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 h = cswap(*(const u32x4*)(Cs + row * lds_s + blk * 32 + q * 8), row);
        pp[4 * q] = h[0]; pp[4 * q + 1] = h[1]; pp[4 * q + 2] = h[2]; pp[4 * q + 3] = h[3];
      }
      unsigned w[8];
      const int ex = mx_block_pk(pp, w);
      unsigned char* dst = qr + (m0 + row) * N + n0 + blk * 32;
      *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
      *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
      sr[(m0 + row) * (N / 32) + n0 / 32 + blk] = (unsigned char)(ex + 127);
    }
  }
  constexpr int NP = BN / 2, RGN = BM / 32, CBLK = NP * RGN;
  static_assert(RGN % 4 == 0 && NP % 16 == 0 && NT % 64 == 0, "MX column pass: 4 row groups x 16 column pairs per wave");
#pragma unroll
  for (int k0 = 0; k0 < CBLK; k0 += NT) {
    const int k = k0 + tid, q = k >> 6, l = k & 63;
    const int rg = (q % (RGN / 4)) * 4 + (l >> 4), cp = (q / (RGN / 4)) * 16 + (l & 15), col = 2 * cp;
    if (k < CBLK && col < cols && rg * 32 < rows) {
      unsigned lo[16], hi[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ra = rg * 32 + 2 * r, rb = ra + 1;
        const unsigned a = *(const unsigned*)(Cs + ra * lds_s + (col ^ cswz(ra)));
        const unsigned b = *(const unsigned*)(Cs + rb * lds_s + (col ^ cswz(rb)));
        lo[r] = __builtin_amdgcn_perm(b, a, 0x05040100u);
        hi[r] = __builtin_amdgcn_perm(b, a, 0x07060302u);
      }
      unsigned w[8];
      int ex = mx_block_pk(lo, w);
      unsigned char* dst = qc + (n0 + col) * M + m0 + rg * 32;
      *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
      *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
      sc[(n0 + col) * (M / 32) + m0 / 32 + rg] = (unsigned char)(ex + 127);
      ex = mx_block_pk(hi, w);
      dst += M;
      *(u32x4*)dst = u32x4{w[0], w[1], w[2], w[3]};
      *(u32x4*)(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
      sc[(n0 + col + 1) * (M / 32) + m0 / 32 + rg] = (unsigned char)(ex + 127);
    }
  }
}

// LDS the bf16 epilogues need: the padded C tile + the [2][WM][BN] f32 BN-statistics partials.
template <int BM, int BN, int WM>
constexpr int epi_lds_bytes() { return BM * (BN + 8) * 2 + 2 * WM * BN * 4; }

// DPP row rotate (16-lane rows); rotates stay inside the row so every source lane is valid.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes of a DPP row; every lane of the row gets the total (VALU only, no LDS).
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f32<0x128>(v);  // row_ror:8
  v += dpp_f32<0x124>(v);  // row_ror:4
  v += dpp_f32<0x122>(v);  // row_ror:2
  v += dpp_f32<0x121>(v);  // row_ror:1
  return v;
}

// Relu keep-bits of an 8-column pre-activation chunk (bit e = v[e] > 0): the EXT epilogue's aux_bits.
__device__ __forceinline__ unsigned char relu_bits8(bf16x8 v) {
  unsigned b = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) b |= (bf2f(v[e]) > 0.f ? 1u : 0u) << e;
  return (unsigned char)b;
}

// Output row of GEMM row m under the out-map (identity without one).
__device__ __forceinline__ long long out_row(const GemmParams& p, int m) {
  if (p.om_hp == 0) return m;
  const int hw = p.om_hp * p.om_wp;
  const int n = m / hw, rem = m - n * hw, h = rem / p.om_wp, w = rem - h * p.om_wp;
  return ((long long)n * p.om_h + h * p.om_sh + p.om_a) * p.om_w + w * p.om_sw + p.om_b;
}
// Residual row of output row mo (-1: off the sub-sampling lattice -> no residual).
__device__ __forceinline__ long long resid_row(const GemmParams& p, long long mo) {
  if (p.rs_sh == 0) return mo;
  const long long hw = (long long)p.rs_h * p.rs_w;
  const long long n = mo / hw;
  const int rem = (int)(mo - n * hw), h = rem / p.rs_w, w = rem - h * p.rs_w;
  if (h % p.rs_sh != 0 || w % p.rs_sw != 0) return -1;
  return (n * p.rs_p + h / p.rs_sh) * p.rs_q + w / p.rs_sw;
}

// DRAIN: the caller has LDS-DMA loads in flight (persistent g4: the next tile's prefetch), which
// the compiler's vmcnt bookkeeping does not model -- wait for all of them before the store pass
// issues its own global loads (residual, BN-reduce inputs), so those waits stay exact.
// QUAD: the 8-phase engine's wave layout (gemm_g8.hip): wave (wm, wn) owns the four quadrant
// sub-tiles rows {q*BM/2 + wm*64 + [0,64)} x cols {q'*BN/2 + wn*32 + [0,32)}; row fragment i covers
// rows (i>>2)*BM/2 + wm*64 + (i&3)*16, column fragment j cols (j>>1)*BN/2 + wn*32 + (j&1)*16.
template <int BM, int BN, int NT, int WM, int EPI, int BNRG = 0, bool DRAIN = false, bool QUAD = false>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, f32x4 (&acc)[BM / WM / 16][BN / (NT / 64 / WM) / 16],
                                              char* smem, int m0, int n0, int bz) {
  constexpr int NW = NT / 64, WN = NW / WM;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ml = lane & 15, nl = (lane >> 4) * 4;
  static_assert(!QUAD || (FM == 8 && FN == 4), "QUAD: 8 row x 4 column fragments per wave");
  auto frow = [&](int i) { return QUAD ? (i >> 2) * (BM / 2) + wm * 64 + (i & 3) * 16 : wm * TM + i * 16; };
  auto fcol = [&](int j) { return QUAD ? (j >> 1) * (BN / 2) + wn * 32 + (j & 1) * 16 : wn * TN + j * 16; };
  constexpr bool ext = (EPI == EPI_BF16_EXT || EPI == EPI_BF16_EXT_MX), mx = (EPI == EPI_BF16_EXT_MX);
  if constexpr (EPI == EPI_F32) {
    // split_stride < 0: every split adds its partial straight into C with hardware f32 atomics
    // (global_atomic_add_f32, -munsafe-fp-atomics) -- no slab workspace, no reduce pass.
    const bool atomic = p.split_stride < 0;
    float* C = (float*)p.C + bz * p.sC + (atomic ? 0LL : (long long)blockIdx.z * p.split_stride);
    // interior tile, plain store (the split-K slabs of every weight gradient): no per-element
    // bounds, atomic or beta checks (each compiled to a compare and an exec-masked branch)
    if (!atomic && p.beta == 0.f && m0 + BM <= p.M && n0 + BN <= p.N && (p.ldc & 3) == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          *(f32x4*)(C + (long long)(m0 + frow(i) + ml) * p.ldc + n0 + fcol(j) + nl) = acc[i][j] * p.alpha;
      return;
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = m0 + frow(i) + ml;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + fcol(j) + nl;
        float* dst = C + (long long)m * p.ldc + n;
        f32x4 v = acc[i][j] * p.alpha;
        if (atomic) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) atomicAdd(dst + r, v[r]);
        } else if (n + 3 < p.N && (p.ldc & 3) == 0) {
          if (p.beta != 0.f) v += p.beta * *(f32x4*)dst;
          *(f32x4*)dst = v;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = v[r] + (p.beta != 0.f ? p.beta * dst[r] : 0.f);
        }
      }
    }
  } else {
    constexpr int LDC_S = BN + 8;  // padded bf16 row stride of the LDS C tile
    bf16* Cs = (bf16*)smem;
    // element offset of logical (row, col) in the swizzled C tile; cbase: a 16-B chunk's slot (col % 8 == 0)
    auto cso = [&](int row, int col) { return row * LDC_S + (col ^ cswz(row)); };
    auto cbase = [&](int row, int col8) { return row * LDC_S + col8; };
    float csum[FN][4], csq[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { csum[j][r] = 0.f; csq[j][r] = 0.f; }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nloc = fcol(j) + nl;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (n0 + nloc + r < p.N) ? p.bias[n0 + nloc + r] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int mloc = frow(i) + ml;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] * p.alpha + bv[r];
          if constexpr (EPI == EPI_BF16_ACT) v = act_apply(v, p.act);  // EXT: in the store pass
          csum[j][r] += v;
          csq[j][r] += v * v;
          o[r] = f2bf(v);
        }
        *(bf16x4*)(Cs + cso(mloc, nloc)) = o;
      }
    }
    // BN batch statistics (rows >= M were zero-filled -> contribute 0; no bias in conv use):
    // 16-lane row sums by DPP, the WM waves of a column meet in LDS behind the C tile, then ONE
    // coalesced atomic per (column, stat) per block instead of 4-lane atomics per wave.
    float* red = (float*)(smem + BM * LDC_S * 2);  // [2][WM][BN]
    if (p.stats) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s = row16_sum(csum[j][r]), q = row16_sum(csq[j][r]);
          if (ml == 0) {
            const int nloc = fcol(j) + nl + r;
            red[wm * BN + nloc] = s;
            red[(WM + wm) * BN + nloc] = q;
          }
        }
    }
    __syncthreads();
    if (p.stats) {
      float* st = p.stats + (long long)(blockIdx.x % p.stats_shards) * 2 * p.N;
      for (int t = tid; t < 2 * BN; t += NT) {
        const int w = t / BN, col = t - w * BN, n = n0 + col;
        if (n < p.N) {
          float v = 0.f;
#pragma unroll
          for (int k = 0; k < WM; ++k) v += red[(w * WM + k) * BN + col];
          atomicAdd(st + (long long)w * p.N + n, v);
        }
      }
    }
    bf16* C = (bf16*)p.C + bz * p.sC;
    constexpr int CPR = BN / 8, TOT = BM * CPR;
    constexpr bool bnr = (EPI == EPI_BF16_BNR);
    const int ccol = tid % CPR;  // this thread's 8-column chunk (fixed: NT % CPR == 0)
    // BN-reduce partials: r0 = sum dz, r1 = sum dz*y, r2 = sum dz*y2 over this thread's chunks;
    // the centring (y - mean) * invstd is applied once after the loop (r1 <- (r1 - mean*r0) *
    // invstd), so mean/invstd need no registers inside the store pass -- those 32 VGPRs pay for a
    // second chunk in flight on the 128-VGPR (4 waves/SIMD) instantiations.
    // (the relu-from-y mask's scale/shift are re-read per chunk from L1/L2 instead of pinning 16
    // VGPRs for the whole store pass)
    float r0[8], r1[8], r2[8];
    if constexpr (bnr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) r0[e] = r1[e] = r2[e] = 0.f;
    }
    // Interior tile (block-uniform): the store pass runs in groups of G chunks whose global loads
    // (residual, BN inputs, activation-backward source) are ALL issued before the group's first
    // store. Written load -> store per chunk, the compiler cannot hoist the next chunk's loads over
    // a store that may alias them, and every chunk paid two full memory latencies (vmcnt(0) before
    // and after its store: measured 3 TB/s on the BN-backward dgrads). Loads are unconditional from
    // always-valid addresses (absent tensors alias y / C) so no per-element branch splits them.
    if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool tile_fast = (m0 + BM <= p.M) && (n0 + BN <= p.N) && ((p.ldc & 7) == 0);
    constexpr int NIT = TOT / NT;
    // BNR groups: BNRG chunks in flight (the caller sizes it to its VGPR budget; 0 -> 1). Measured
    // on the 128-VGPR single-stage 128x128 kernels (ResNet-50 bs256 step): 1 -> 26.47 ms, 2 -> 26.32,
    // 4 -> 29.52 (208 B/lane of spills). Every
    // load below is from an in-bounds address: absent tensors are not loaded at all (block-uniform
    // branches), and off the residual lattice the (unused) residual load reads C.
    // EXT groups of 4 (2 until round 6: with the per-element activation switches gone they fit;
    // BERT-base 9.95 -> 9.89 ms, Transformer-big 16.93 -> 16.85); plain groups of 8 measured level.
    constexpr int GB = BNRG > 0 ? BNRG : 1;
    constexpr int GCAP = bnr ? GB : 4;
    constexpr int G = NIT < GCAP ? NIT : GCAP;
    if (tile_fast) {
      const bf16* resid_b = p.resid ? (const bf16*)p.resid : (const bf16*)p.C;
      const bf16* dsrc_b = (ext && p.dact_src) ? (const bf16*)p.dact_src : (const bf16*)p.C;
      const bf16* y_b = bnr ? (const bf16*)p.bn_y : nullptr;
      const bf16* y2_b = bnr ? (p.bn_y2 ? (const bf16*)p.bn_y2 : y_b) : nullptr;
      const unsigned char* mk_b = bnr ? (p.bn_amask ? p.bn_amask : (const unsigned char*)y_b) : nullptr;
      // one group of GS chunks whose loads are all issued before its first store
      auto group = [&](auto gsz, int g0) {
        constexpr int GS = decltype(gsz)::value;
        bf16x8 cv[GS], rr[GS], zv[GS], yv[GS], y2v[GS];
        unsigned mk[GS], zb[GS];
        long long off[GS];
        bool rok[GS];
        int mlog[GS], nlog[GS], lofs[GS], lrow[GS];
#pragma unroll
        for (int g = 0; g < GS; ++g) {
          const int idx = tid + (g0 + g) * NT;
          const int row = idx / CPR, cc = idx - row * CPR;
          lofs[g] = cbase(row, cc * 8);
          lrow[g] = row;
          const int m = m0 + row, n = n0 + cc * 8;
          long long mo = m, mr = m;
          if constexpr (bnr) { mo = out_row(p, m); mr = resid_row(p, mo); }
          off[g] = bz * p.sC + mo * p.ldc + n;
          rok[g] = p.resid && mr >= 0;
          mlog[g] = m; nlog[g] = n;
          cv[g] = crd8(Cs + lofs[g], row);
          // off the residual's sub-sampling lattice the (unused) load reads C itself: resid is the
          // smaller lattice tensor there, so resid + off[g] could run past its allocation
          if (p.resid) rr[g] = *(const bf16x8*)(rok[g] ? resid_b + bz * p.sC + mr * p.ldc + n : (const bf16*)p.C + off[g]);
          if constexpr (ext) {
            if (p.dact_src) {
              if (p.dact_bits) zb[g] = ((const unsigned char*)p.dact_src)[off[g] >> 3];
              else zv[g] = *(const bf16x8*)(dsrc_b + off[g]);
            }
          }
          if constexpr (bnr) {
            yv[g] = *(const bf16x8*)(y_b + off[g]);
            if (p.bn_amask) mk[g] = mk_b[off[g] >> 3];
            if (p.bn_y2) y2v[g] = *(const bf16x8*)(y2_b + off[g]);
          }
        }
#pragma unroll
        for (int g = 0; g < GS; ++g) {
          bf16x8 v = cv[g];
          if constexpr (ext) {
            // pre-activation chunk: [* act'(z)] -> [aux copy] -> act -> [dropout]
            float f[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = bf2f(v[e]);
            if (p.dact_src) {
              if (p.dact_bits) {
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] = (zb[g] >> e) & 1u ? f[e] : 0.f;
              } else {
                act_grad_mul8(f, zv[g], p.dact);
              }
            }
            if (p.aux) {
              if (p.aux_bits) ((unsigned char*)p.aux)[off[g] >> 3] = relu_bits8(v);
              else *(bf16x8*)((bf16*)p.aux + off[g]) = v;
            }
            act_apply8(f, p.act);
            if (p.drop_p > 0.f) {
              const unsigned long long lin = (unsigned long long)mlog[g] * p.N + nlog[g];
              const unsigned km = drop_keep8(drop_seed32(eff_seed(p.drop_seed, p.drop_seed_key)), lin, drop_thr8(p.drop_p));
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] = (km >> e) & 1u ? f[e] * p.drop_scale : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = f2bf(f[e]);
          }
          if (rok[g]) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(rr[g][e]));
          }
          // relu keep-bits of the chunk (one VGPR); store_dz masks v with them before the store
          unsigned keepm = 0xffu;
          if constexpr (bnr) {
            if (p.bn_amask) {
              keepm = mk[g];
            } else if (p.bn_relu) {
              keepm = 0;
              const f32x4* scp = (const f32x4*)(p.bn_scale + nlog[g]);
              const f32x4* shp = (const f32x4*)(p.bn_shift + nlog[g]);
              const f32x4 s0 = scp[0], s1 = scp[1], h0 = shp[0], h1 = shp[1];
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float scl = e < 4 ? s0[e & 3] : s1[e & 3], shf = e < 4 ? h0[e & 3] : h1[e & 3];
                keepm |= (bf2f(yv[g][e]) * scl + shf > 0.f) ? (1u << e) : 0u;
              }
            }
            if (p.bn_store_dz) {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (!((keepm >> e) & 1u)) v[e] = f2bf(0.f);
            }
          }
          if constexpr (mx) {
            cwr8(Cs + lofs[g], v, lrow[g]);  // the final value, for the MX pass
            if (!p.mx_skip_c) *(bf16x8*)((bf16*)p.C + off[g]) = v;
          } else {
            if constexpr (ext) {
              if (p.colsum) cwr8(Cs + lofs[g], v, lrow[g]);  // the final value, for the column sums
            }
            *(bf16x8*)((bf16*)p.C + off[g]) = v;
          }
          if constexpr (bnr) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float y = bf2f(yv[g][e]);
              const float dz = ((keepm >> e) & 1u) ? bf2f(v[e]) : 0.f;
              r0[e] += dz;
              r1[e] += dz * y;
              if (p.bn_y2) r2[e] += dz * bf2f(y2v[g][e]);
            }
          }
        }
            };
      // full groups of G chunks (rolled for BNR: VGPR budget), then a compile-time remainder group
      // when G does not divide NIT (the halo conv's tiles: NIT = 7)
      constexpr int NF = NIT / G, REM = NIT - NF * G;
#pragma unroll (bnr ? 1 : NF)
      for (int k = 0; k < NF; ++k) group(std::integral_constant<int, G>{}, k * G);
      if constexpr (REM > 0) group(std::integral_constant<int, REM>{}, NF * G);
    } else {
#pragma unroll 1
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NT;
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row, n = n0 + cc * 8;
      if (m >= p.M || n >= p.N) continue;
      // row maps (strided-conv dgrad) exist on the BN-backward epilogue only: elsewhere they would
      // cost registers the persistent kernels do not have
      long long mo = m, mr = m;
      if constexpr (bnr) { mo = out_row(p, m); mr = resid_row(p, mo); }
      const bf16* rsrc = (p.resid && mr >= 0) ? (const bf16*)p.resid + bz * p.sC + mr * p.ldc + n : nullptr;
      bf16x8 v = crd8(Cs + cbase(row, cc * 8), row);
      bf16* dst = C + mo * p.ldc + n;
      if (n + 7 < p.N && (p.ldc & 7) == 0) {
        const long long off = bz * p.sC + mo * p.ldc + n;
        if constexpr (ext) {
          // pre-activation chunk: [* act'(z)] -> [aux copy] -> act -> [dropout]; 16-B coalesced
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = bf2f(v[e]);
          if (p.dact_src) {
            if (p.dact_bits) {
              const unsigned zb = ((const unsigned char*)p.dact_src)[off >> 3];
#pragma unroll
              for (int e = 0; e < 8; ++e) f[e] = (zb >> e) & 1u ? f[e] : 0.f;
            } else {
              const bf16x8 zv = *(const bf16x8*)((const bf16*)p.dact_src + off);
              act_grad_mul8(f, zv, p.dact);
            }
          }
          if (p.aux) {
            if (p.aux_bits) ((unsigned char*)p.aux)[off >> 3] = relu_bits8(v);
            else *(bf16x8*)((bf16*)p.aux + off) = v;
          }
          act_apply8(f, p.act);
          if (p.drop_p > 0.f) {
            const unsigned long long lin = (unsigned long long)m * p.N + n;
            const unsigned km = drop_keep8(drop_seed32(eff_seed(p.drop_seed, p.drop_seed_key)), lin, drop_thr8(p.drop_p));
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = (km >> e) & 1u ? f[e] * p.drop_scale : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(f[e]);
        }
        if (rsrc) {
          bf16x8 rr = *(const bf16x8*)rsrc;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + bf2f(rr[e]));
        }
        if constexpr (bnr) {
          bf16x8 yv = *(const bf16x8*)((const bf16*)p.bn_y + off);
          bf16x8 y2v;
          if (p.bn_y2) y2v = *(const bf16x8*)((const bf16*)p.bn_y2 + off);
          const unsigned mk = p.bn_amask ? p.bn_amask[off >> 3] : 0xffu;
          unsigned keepm = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float y = bf2f(yv[e]);
            bool keep = p.bn_amask ? ((mk >> e) & 1u) != 0
                                   : (p.bn_relu ? (y * p.bn_scale[n + e] + p.bn_shift[n + e] > 0.f) : true);
            keepm |= keep ? (1u << e) : 0u;
            const float dz = keep ? bf2f(v[e]) : 0.f;
            r0[e] += dz;
            r1[e] += dz * y;
            if (p.bn_y2) r2[e] += dz * bf2f(y2v[e]);
          }
          if (p.bn_store_dz) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (!((keepm >> e) & 1u)) v[e] = f2bf(0.f);
          }
        }
        if constexpr (mx) {
          cwr8(Cs + cbase(row, cc * 8), v, row);
          if (!p.mx_skip_c) *(bf16x8*)dst = v;
        } else {
          if constexpr (ext) {
            if (p.colsum) cwr8(Cs + cbase(row, cc * 8), v, row);
          }
          *(bf16x8*)dst = v;
        }
      } else {
        unsigned abits = 0;
        for (int e = 0; e < 8 && n + e < p.N; ++e) {
          const long long off = bz * p.sC + mo * p.ldc + n + e;
          float x = bf2f(v[e]);
          if constexpr (ext) {
            if (p.dact_src) {
              if (p.dact_bits) x = (((const unsigned char*)p.dact_src)[off >> 3] >> e) & 1u ? x : 0.f;
              else x *= act_grad(bf2f(((const bf16*)p.dact_src)[off]), p.dact);
            }
            if (p.aux) {
              if (p.aux_bits) abits |= (bf2f(v[e]) > 0.f ? 1u : 0u) << e;
              else ((bf16*)p.aux)[off] = v[e];
            }
            x = act_apply(x, p.act);
            if (p.drop_p > 0.f)
              x = drop_keep1(drop_seed32(eff_seed(p.drop_seed, p.drop_seed_key)), (unsigned long long)m * p.N + n + e, drop_thr8(p.drop_p)) ? x * p.drop_scale : 0.f;
            x = bf2f(f2bf(x));
          }
          if (rsrc) x += bf2f(rsrc[e]);
          dst[e] = f2bf(x);
          if constexpr (ext) {
            if (p.colsum) Cs[cso(row, cc * 8 + e)] = f2bf(x);
          }
        }
        if constexpr (ext) {
          if (p.aux && p.aux_bits) ((unsigned char*)p.aux)[(bz * p.sC + mo * p.ldc + n) >> 3] = (unsigned char)abits;
        }
      }
    }
    }  // ragged tile
    if constexpr (ext) {
      // p.colsum += column sums of the final tile (the LDS C tile holds every final value now):
      // RG row groups per column -> partials in the reduction area behind the tile -> one global
      // f32 atomic per column per block
      if (p.colsum) {
        constexpr int RG = NT >= BN ? NT / BN : 1;
        float* part = (float*)(smem + BM * LDC_S * 2);  // [RG][BN] (<= [2][WM][BN])
        static_assert(RG * BN <= 2 * WM * BN, "column-sum partials fit the reduction area");
        const int rows = min(BM, p.M - m0), cols = min(BN, p.N - n0);
        __syncthreads();
        for (int t = tid; t < RG * BN; t += NT) {
          const int rg = t / BN, col = t - rg * BN;
          float a = 0.f;
          if (col < cols)
            for (int r = rg; r < rows; r += RG) a += bf2f(Cs[cso(r, col)]);
          part[rg * BN + col] = a;
        }
        __syncthreads();
        for (int col = tid; col < cols; col += NT) {
          float a = 0.f;
#pragma unroll
          for (int rg = 0; rg < RG; ++rg) a += part[rg * BN + col];
          atomicAdd(p.colsum + n0 + col, a);
        }
      }
    }
    if constexpr (mx) {
      __syncthreads();  // every final chunk is in the LDS tile
      mx_tile_out<BM, BN, NT>(p, Cs, LDC_S, m0, n0);
    }
    if constexpr (bnr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int n = min(n0 + ccol * 8 + e, p.N - 1);
        r1[e] = (r1[e] - p.bn_mean[n] * r0[e]) * p.bn_invstd[n];
        if (p.bn_y2) r2[e] = (r2[e] - p.bn_mean2[n] * r0[e]) * p.bn_invstd2[n];
      }
      // lanes sharing a column chunk: tid % CPR equal -> xor over the bits above log2(CPR)
      // (DPP / permlane-swap butterflies: no LDS round trip per step)
      static_assert(CPR >= 8, "BN-reduce lane butterfly needs >= 8 chunks per row");
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (CPR <= 8) { r0[e] = xor_sum<8>(r0[e]); r1[e] = xor_sum<8>(r1[e]); r2[e] = xor_sum<8>(r2[e]); }
        if constexpr (CPR <= 16) { r0[e] = xor_sum<16>(r0[e]); r1[e] = xor_sum<16>(r1[e]); r2[e] = xor_sum<16>(r2[e]); }
        if constexpr (CPR <= 32) { r0[e] = xor_sum<32>(r0[e]); r1[e] = xor_sum<32>(r1[e]); r2[e] = xor_sum<32>(r2[e]); }
      }
      __syncthreads();  // C tile no longer needed: reuse LDS for the cross-wave reduction
      float* red = (float*)smem;  // [NW waves][3][CPR*8]
      if (lane < CPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[(wid * 3 + 0) * (CPR * 8) + lane * 8 + e] = r0[e];
          red[(wid * 3 + 1) * (CPR * 8) + lane * 8 + e] = r1[e];
          red[(wid * 3 + 2) * (CPR * 8) + lane * 8 + e] = r2[e];
        }
      }
      __syncthreads();
      const int nsum = p.bn_y2 ? 3 : 2;
      float* st = p.bn_sums + (long long)(blockIdx.x % p.bn_shards) * 3 * p.N;
      for (int k = tid; k < nsum * CPR * 8; k += NT) {
        const int which = k / (CPR * 8), col = k - which * (CPR * 8);
        const int n = n0 + col;
        if (n >= p.N) continue;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[(w * 3 + which) * (CPR * 8) + col];
        atomicAdd(st + which * p.N + n, v);
      }
    }
  }
}

}  // namespace tfk
