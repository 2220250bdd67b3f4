"""LDS-DMA intake per CU versus bytes in flight (ldsdma_rate.hip): for each ring (slots x tile
KiB x waves) and source (L2-resident window / HBM sweep), the median per-workgroup rate and
the chip-wide rate. Usage: python bench/probes/ldsdma_rate.py [--build]"""
import argparse
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "ldsdma_rate.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared",
                           "-fPIC", "-o", SO, os.path.join(HERE, "ldsdma_rate.hip")])


CFGS = [(2, 16, 4), (3, 16, 4), (4, 16, 4), (6, 16, 4), (8, 16, 4), (2, 32, 4), (3, 32, 4),
        (4, 32, 4), (2, 32, 8), (3, 32, 8), (4, 32, 8), (5, 32, 8), (2, 64, 8), (2, 48, 8),
        (3, 48, 8), (10, 16, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    if a.build or not os.path.exists(SO):
        build()
    lib = ctypes.CDLL(SO)
    lib.ldsdma_probe.restype = ctypes.c_int
    lib.ldsdma_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda")
    big = torch.ones(3 << 30, dtype=torch.uint8, device=dev)  # 3 GiB: HBM sweep
    out = torch.zeros(4096, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for ns, kb, nw in CFGS:
        lds_kb = ns * kb
        per_cu = max(1, min(160 // lds_kb, 8))
        for sweep in (0, 1):
            for wpc in sorted({1, per_cu}):
                wgs = 256 * wpc
                steps = a.steps if not sweep else min(a.steps, (3 << 30) // (wgs * kb * 1024) - ns)
                code = ns * 1000 + kb * 10 + nw // 4
                for _ in range(2):  # warm-up + measured
                    rc = lib.ldsdma_probe(code, big.data_ptr(), big.numel(), steps, sweep,
                                          out.data_ptr(), wgs, stream)
                    assert rc == 0, (code, rc)
                    torch.cuda.synchronize()
                t = (out[:wgs] & ((1 << 62) - 1)).double().cpu() / 100.0  # 100 MHz -> us
                med = float(t.median())
                wg_bytes = steps * kb * 1024
                print(json.dumps({"slots": ns, "tile_kb": kb, "waves": nw, "wg_per_cu": wpc,
                                  "src": "hbm" if sweep else "l2", "inflight_kb_per_cu":
                                  (ns - 1) * kb * wpc, "us_med": round(med, 2),
                                  "gbs_per_cu": round(wg_bytes * wpc / med / 1e3, 1),
                                  "chip_tbs": round(wg_bytes * wgs / float(t.max()) / 1e6, 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
