"""Where the headline step's time goes between kernels.

Runs bench.py's headline step (RS(6,4), 4,096 x 64 KiB stripes, encode then
erase-0 decode, 4 rotating batches) for --steps steps per mode and prints the
wall time per step next to the sum of the two kernels' HIP-event times:

  eager      launches only (no events in the stream)
  events     bench.py's form before round 4's fix: 3 torch timing events per step (system-scope release)
  devevents  the same with bench.Event (device-scope release, bench.py's default now)
  graph      one HIP graph per batch (encode + decode), replayed

Run under `rocprofv3 --kernel-trace` to see the gaps themselves.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from elect_amd.batch import decode_batch, encode_batch  # noqa: E402
from elect_amd.coder import RSCoder  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--modes", default="eager,events,devevents,graph,eager,devevents")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    k, m, L, B = 4, 2, 65536, 4096
    coder = RSCoder(k, m)
    g = torch.Generator(device=dev).manual_seed(7)
    sets = []
    for _ in range(4):
        st = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
        st[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
        sets.append((st, torch.empty((B, 1, L), dtype=torch.uint8, device=dev)))
    surv = list(range(1, k + 1))
    ops = [(lambda st=st: encode_batch(coder, st[:, :k], st[:, k:]),
            lambda st=st, rb=rb: decode_batch(coder, st, surv, [0], rb, inputs_by_unit=True)) for st, rb in sets]

    graphs = None
    res = {}
    for mode in args.modes.split(","):
        if mode == "graph" and graphs is None:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for e, d in ops:
                    e(); d()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            graphs = []
            for e, d in ops:
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    e(); d()
                graphs.append(gr)
        mk = bench.Event if mode == "devevents" else (lambda: torch.cuda.Event(enable_timing=True))
        evs = [[mk() for _ in range(3)] for _ in range(args.steps)]
        for i in range(8):
            e, d = ops[i % 4]
            e(); d()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            e, d = ops[i % 4]
            if mode in ("events", "devevents"):
                evs[i][0].record(); e(); evs[i][1].record(); d(); evs[i][2].record()
            elif mode == "graph":
                graphs[i % 4].replay()
            else:
                e(); d()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        r = {"wall_ms_per_step": round(wall, 4)}
        if mode in ("events", "devevents"):
            r["kernels_ms_per_step"] = round(sum(x[0].elapsed_time(x[2]) for x in evs) / args.steps, 4)
            r["between_steps_ms"] = round(sum(evs[i][2].elapsed_time(evs[i + 1][0])
                                              for i in range(args.steps - 1)) / (args.steps - 1), 4)
        res.setdefault(mode, []).append(r)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
