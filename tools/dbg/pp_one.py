"""Run one GEMM shape/direction N times (for rocprofv3 PMC passes)."""
import sys, torch
sys.path.insert(0, '.')
from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops._lib import lib
M, N, K = [int(v) for v in sys.argv[1:4]]
mode = sys.argv[4] if len(sys.argv) > 4 else "fwd"
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
x = (torch.rand(M, K, device='cuda') * 2 - 1).to(torch.bfloat16)
w = (torch.rand(N, K, device='cuda') * 2 - 1).to(torch.bfloat16)
y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
dy = (torch.rand(M, N, device='cuda') * 2 - 1).to(torch.bfloat16)
dx = torch.empty(M, K, device='cuda', dtype=torch.bfloat16)
for _ in range(reps):
    if mode == "fwd":
        G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, (256, 256))
    elif mode == "dgrad":
        G._gemm(dy, w, dx, M, K, N, N, K, K, G.A_KIN, G.B_KOUT, G.EPI_BF16, (256, 256))
    else:
        _ = x @ w.t()
torch.cuda.synchronize()
