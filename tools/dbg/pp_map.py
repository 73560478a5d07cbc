import torch, sys
sys.path.insert(0, '.')
from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops._lib import lib
L = lib()
M = N = 256; K = 64
x = torch.zeros(M, K); x[:, 0] = 1.0  # every row: A[m][0] = 1
w = torch.zeros(N, K); w[:, 0] = torch.arange(N).float()  # C[m][n] = n
x = x.to(torch.bfloat16).cuda(); w = w.to(torch.bfloat16).cuda()
for ext in (0, 1):
    for pp in (1, 0):
        L.gemm_set_pp(pp)
        y = torch.empty(M, N, dtype=torch.bfloat16, device='cuda')
        aux = torch.empty(M, N, dtype=torch.bfloat16, device='cuda') if ext else None
        G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, (256, 256), aux=aux)
        torch.cuda.synchronize()
        print('ext', ext, 'pp', pp, 'row0', y[0, :40].float().tolist())
        print('   row5', y[5, :20].float().tolist())
