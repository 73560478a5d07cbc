// w128 GEMM variant 1 (default scheduler, loop body split at `if (more)`); kernel body: gemm_w128.h
#define W128_NS w128a
#define W128_V2 0
#define W128_SGB 0
#include "gemm_w128.h"

using namespace tfk;

// 0 = off (g4 256x256), 1..4 = variant (TFK_W128=<n> or tfk_w128_set(n); -1 -> back to the env)
static int g_w128 = -1;
static int w128_variant() {
  if (g_w128 < 0) {
    const char* e = getenv("TFK_W128");
    g_w128 = e ? atoi(e) : 0;
  }
  return g_w128;
}
extern "C" void tfk_w128_set(int v) { g_w128 = v < 0 ? -1 : v; }
extern "C" int tfk_w128b_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits, hipStream_t stream);
extern "C" int tfk_w128c_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits, hipStream_t stream);
extern "C" int tfk_w128d_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits, hipStream_t stream);

#define W128_CASE(AM_, BM2_, EPI_)                                                                 \
  if (amode == AM_ && bmode == BM2_ && epi == EPI_) {                                              \
    hipLaunchKernelGGL((w128a::w128_kernel<AM_, BM2_, EPI_>), dim3(tiles, batch, splits),            \
                       dim3(w128a::NTH), 0, stream, p);                                             \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                               \
  }
// p.tiles_n / p.kt_per_split already set for 256x256 tiles by the caller (tfk_g4_launch)
extern "C" int tfk_w128a_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits,
                              hipStream_t stream) {
  W128_CASE(0, 0, EPI_BF16)
  W128_CASE(0, 0, EPI_F32)
  W128_CASE(0, 1, EPI_BF16)
  W128_CASE(0, 1, EPI_F32)
  W128_CASE(1, 1, EPI_F32)
  W128_CASE(1, 1, EPI_BF16)
  return -1;
}

// Dense 256x256 GEMMs (g4 operand modes KIN/KOUT, no conv gather) on the selected variant.
// Returns -1 when off / not instantiated (the caller falls back to g4).
extern "C" int tfk_w128_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits,
                               hipStream_t stream) {
  const int v = w128_variant();
  if (v <= 0 || amode == 2 || bmode == 2) return -1;
  switch (v) {
    case 1: return tfk_w128a_launch(p, amode, bmode, epi, tiles, batch, splits, stream);
    case 2: return tfk_w128b_launch(p, amode, bmode, epi, tiles, batch, splits, stream);
    case 3: return tfk_w128c_launch(p, amode, bmode, epi, tiles, batch, splits, stream);
    case 4: return tfk_w128d_launch(p, amode, bmode, epi, tiles, batch, splits, stream);
  }
  return -1;
}
