import sys, time, json, torch
sys.path.insert(0, '.')
from tensorflow_k8s_amd.ops import fp8 as F8
from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops._lib import lib
for name, (M, N, K) in {"tfm_ffn1": (16384, 4096, 1024), "tfm_ffn2": (16384, 1024, 4096), "tfm_logits": (8192, 33728, 1024), "bert_ffn1": (8192, 3072, 768), "sq8192": (8192, 8192, 8192)}.items():
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16); w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    xq, wq = F8.mx_quantize(x), F8.mx_quantize(w)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    row = {"shape": name}
    for eng in (1, 0):
        lib().fp8_set_engine(eng)
        f = lambda: lib().gemm_mxfp8(xq[0], xq[1], wq[0], wq[1], y, M, N, K, None, None, 0, None, 0.0, 0)
        f(); torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(20): f()
        torch.cuda.synchronize(); row[f"fp8_{'g4' if eng else 'reg'}_tflops"] = round(2 * M * N * K / ((time.perf_counter() - t0) / 20) / 1e12, 1)
    f = lambda: G.linear_fwd(x, w, out=y)
    f(); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(20): f()
    torch.cuda.synchronize(); row["bf16_g4_tflops"] = round(2 * M * N * K / ((time.perf_counter() - t0) / 20) / 1e12, 1)
    print(json.dumps(row), flush=True)
