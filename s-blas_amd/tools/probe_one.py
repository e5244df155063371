#!/usr/bin/env python3
"""One HBM probe configuration (sblas_hbm_probe) for counter passes:
  python probe_one.py [--mode 4] [--wg 2] [--gib 4] [--reps 4]
modes: 0 read, 1 nt read, 2 copy, 3 blocked read, 4 blocked nt read."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=4)
    ap.add_argument("--wg", type=int, default=2)
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import torch
    import sblas
    nbytes = a.gib << 30
    src = torch.ones(nbytes // 8, dtype=torch.float64, device="cuda")
    dst = torch.zeros(nbytes // 8 if a.mode == 2 else 1, dtype=torch.float64, device="cuda")
    ts = [sblas.hbm_probe_timed(a.mode, src.data_ptr(), dst.data_ptr(), nbytes, a.wg) for _ in range(a.reps)]
    print(f"probe mode {a.mode} wg/CU {a.wg}: {min(ts):.3f} ms = {nbytes / min(ts) / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
