#!/usr/bin/env python3
"""Host link ceiling for the scan pipeline: pinned H2D, D2H and both at once
(two streams), in chunks of --mb MiB, on cuda:0.  Run with HSA_ENABLE_SDMA=0
to compare the blit-kernel copy path against the SDMA engines.
    python scripts/pcie_bw.py [--mb 64] [--reps 40]"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    n = a.mb << 20
    dev = torch.device("cuda", 0)
    h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_src = torch.empty(n, dtype=torch.uint8, device=dev)
    d_dst = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(h2d, d2h):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            if h2d:
                with torch.cuda.stream(s1):
                    d_dst.copy_(h_src, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h_dst.copy_(d_src, non_blocking=True)
        torch.cuda.synchronize()
        return n * a.reps / (time.perf_counter() - t0) / 1e9

    run(True, True)
    print(f"chunk {a.mb} MiB: H2D {run(True, False):.1f} GB/s, D2H {run(False, True):.1f} GB/s, "
          f"both at once {run(True, True):.1f} GB/s each way", flush=True)


if __name__ == "__main__":
    main()
