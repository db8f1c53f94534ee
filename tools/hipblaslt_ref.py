#!/usr/bin/env python
"""Vendor-library reference for the projection GEMMs' k loop: torch._int_mm (int8 x int8 ->
int32, hipBLASLt on ROCm) at the ViT-Base B = 256 shapes, timed with HIP events over
back-to-back launches.  No epilogue (int32 outputs: 4 bytes per element written, where k_pg
writes 1, or reads + writes 8 for the residual ones), so it bounds what a library k loop gets
on the same operands; compare with tools/pg_micro.py's k_pg times and its no-epilogue
diagnostic builds.  Not product code: PyTorch is used here only as the library's launcher."""
import torch

M = 256 * 197
SHAPES = {"qkv": (2304, 768), "out": (768, 768), "up": (3072, 768), "down": (768, 3072)}
PEAK = 256 * 2.4e9 * 8192 / 1e12
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for name, (N, K) in SHAPES.items():
    a = torch.randint(-128, 128, (M, K), dtype=torch.int8, device=dev, generator=g)
    bt = torch.randint(-128, 128, (N, K), dtype=torch.int8, device=dev, generator=g)
    res = {}
    for lay, b in (("b=Bt.T", bt.t()), ("b=contig", bt.t().contiguous())):
        try:
            out = torch._int_mm(a, b)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(3):
                e0.record()
                for _ in range(20):
                    torch._int_mm(a, b)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
            ok = bool(torch.equal(out[:64].cpu(), (a[:64].cpu().to(torch.int64) @ bt.cpu().to(torch.int64).t()).to(torch.int32)))
            res[lay] = f"{best:7.1f} us ({2 * M * N * K / best / 1e6 / PEAK * 100:4.1f}% of int8 peak, rows ok {ok})"
        except Exception as ex:  # noqa: BLE001
            res[lay] = f"error {type(ex).__name__}: {str(ex)[:120]}"
    print(f"{name:5s} M={M} N={N} K={K}: " + "; ".join(f"{k} {v}" for k, v in res.items()), flush=True)
