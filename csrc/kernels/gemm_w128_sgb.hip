// w128 GEMM variant 4 (single-basic-block body + explicit sched_group_barrier pipeline); kernel body: gemm_w128.h
#define W128_NS w128d
#define W128_V2 1
#define W128_SGB 1
#include "gemm_w128.h"

using namespace tfk;


#define W128_CASE(AM_, BM2_, EPI_)                                                                 \
  if (amode == AM_ && bmode == BM2_ && epi == EPI_) {                                              \
    hipLaunchKernelGGL((w128d::w128_kernel<AM_, BM2_, EPI_>), dim3(tiles, batch, splits),            \
                       dim3(w128d::NTH), 0, stream, p);                                             \
    return hipGetLastError() == hipSuccess ? 0 : -2;                                               \
  }
// p.tiles_n / p.kt_per_split already set for 256x256 tiles by the caller (tfk_g4_launch)
extern "C" int tfk_w128d_launch(const GemmParams& p, int amode, int bmode, int epi, int tiles, int batch, int splits,
                              hipStream_t stream) {
  W128_CASE(0, 0, EPI_BF16)
  W128_CASE(0, 0, EPI_F32)
  W128_CASE(0, 1, EPI_BF16)
  W128_CASE(0, 1, EPI_F32)
  W128_CASE(1, 1, EPI_F32)
  W128_CASE(1, 1, EPI_BF16)
  return -1;
}
