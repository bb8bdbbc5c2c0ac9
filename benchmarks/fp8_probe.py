"""Probe hipBLASLt fp8 GEMMs via torch._scaled_mm on gfx950 (OCP e4m3fn), vs bf16 matmul."""
import json
import torch

def t(fn, it=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it

for (M, N, K) in [(16384, 2560, 2048), (16384, 11264, 2048), (16384, 2048, 5632), (16384, 2048, 2048), (65536, 2304, 768)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    tb = t(lambda: a @ b.t())
    res = {"shape": [M, N, K], "bf16_tflops": round(2 * M * N * K / tb / 1e9, 1)}
    try:
        a8 = a.to(torch.float8_e4m3fn)
        b8 = b.to(torch.float8_e4m3fn)
        one = torch.ones((), device="cuda")
        f = lambda: torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        y = f()
        err = ((y.float() - (a8.float() @ b8.float().t())).abs().max() / (a8.float() @ b8.float().t()).abs().max()).item()
        t8 = t(f)
        res.update(fp8_tflops=round(2 * M * N * K / t8 / 1e9, 1), fp8_rel_err=err)
    except Exception as ex:  # noqa: BLE001
        res["fp8_error"] = repr(ex)[:300]
    print(json.dumps(res), flush=True)
