"""CPU checks of the GEMM tile picker (no GPU): which tile each ResNet-50 weight-gradient shape gets."""
from tensorflow_k8s_amd.ops import gemm as G


def test_wide_tile_for_cout64_conv_wgrad():
    # stem 7x7x8 (C padded 3 -> 8) -> 64 and stage-1 3x3 64 -> 64 at bs256: M = Cout = 64, long reduction
    assert G.pick_tile(64, 392, splits_ok=True, K=256 * 112 * 112, wide_ok=True) == (64, 256)
    assert G.pick_tile(64, 576, splits_ok=True, K=256 * 56 * 56, wide_ok=True) == (64, 256)
    # without the mode flag (pointwise / other operand modes) the tile is never chosen
    assert G.pick_tile(64, 576, splits_ok=True, K=256 * 56 * 56) != (64, 256)
    # wider outputs keep the square tiles
    assert G.pick_tile(128, 1152, splits_ok=True, K=256 * 28 * 28, wide_ok=True) != (64, 256)
