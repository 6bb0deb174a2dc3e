#!/usr/bin/env python3
"""Host<->device copy ceilings for the host-staged reduction (measurement
tool): 256 MiB page-locked buffers, H2D alone, D2H alone, and both at once on
two streams. Prints one JSON line."""
import json
import time

import torch

S = 256 << 20
REPS = 10
h_in = torch.empty(S, dtype=torch.uint8).pin_memory()
h_out = torch.empty(S, dtype=torch.uint8).pin_memory()
d_a = torch.empty(S, dtype=torch.uint8, device="cuda")
d_b = torch.empty(S, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / REPS


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_in, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_out.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


res = {}
for name, fn in (("h2d", h2d), ("d2h", d2h), ("both", both)):
    t = timed(fn)
    res[name + "_GB_s"] = round(S / t / 1e9, 1)
res["both_GB_s_each_direction"] = res.pop("both_GB_s")
print(json.dumps(res))
