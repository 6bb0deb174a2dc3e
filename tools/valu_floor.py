#!/usr/bin/env python3
"""VALU-issue floor of one kernel's per-element instruction stream: the
kernel's opcode histogram between its first vector load and first vector
store (the per-element body of a grid-stride fold; see STORES), each opcode priced at the
chip-wide saturated rate tools/valu_rate.hip measured for its kind
(profiles/r04/valu/valu_rate.jsonl, 8 waves per SIMD), times the element-waves of
one launch. Measurement tool: the VALU roofline of the long double
every-member fold.
usage: valu_floor.py OBJECT 'KERNEL SUBSTRING' RATES.jsonl ELEMENTS_PER_LAUNCH [STORES]
       valu_floor.py --bench-legs OBJECT RATES.jsonl   (bench.py's long double kernel legs, one JSON dict)
STORES: the body ends at the STORES-th vector store (default 1; the every-
member fold stores each output when its chain ends: one per output)"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_residency as cr  # noqa: E402

from check_residency import LLVM  # noqa: E402  (one LLVM path for both tools)


def kind(op):
    """the probe kind whose measured rate prices this opcode"""
    if re.match(r"v_(add_co|addc_co|sub_co|subb_co|subrev_co|subbrev_co)_u32", op):
        return "v_add_co+v_addc_co"
    if re.match(r"v_(lshlrev|lshrrev|ashrrev)_(b|i)64|v_lshl_add_u64", op):
        return "v_lshlrev_b64"
    if re.match(r"v_cmp_\w+_(u|i)64", op):
        return "v_cmp_gt_u64(sgpr)"
    if op.startswith("v_cndmask") or op.startswith("v_cmp"):
        return "v_cndmask_b32(sgpr mask)"   # lane-mask producers / consumers
    for m in ("v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32"):
        if op.startswith(m):
            return m
    # the rest at the 32-bit add's rate (measured the same in the 4- and
    # 8-byte encodings: v_add_u32_e64 1.03e12, v_mov_b32 1.05e12)
    return "v_add_u32"


def floor(obj, sub, rates_path, elements, stores=1):
    """the record main() prints, as a dict"""
    rates = {}
    for ln in open(rates_path):
        d = json.loads(ln)
        if d["waves_per_simd"] == 8:
            rates[d["kind"]] = d["chip_wave_insts_per_s"]
    with tempfile.TemporaryDirectory() as t:
        co = cr.code_object(obj, t)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", co], capture_output=True, text=True,
                             check=True).stdout.splitlines()
    start = next(i for i, ln in enumerate(dis) if re.match(r"^[0-9a-f]+ <", ln) and sub in ln)
    end = next((i for i in range(start + 1, len(dis)) if re.match(r"^[0-9a-f]+ <", dis[i])), len(dis))
    body = [ln.strip().split("//")[0].split()[0] for ln in dis[start + 1:end] if ln.startswith("\t")]
    lo = next(i for i, op in enumerate(body) if op.startswith(("global_load", "buffer_load")))
    hi = [i for i, op in enumerate(body) if op.startswith(("global_store", "buffer_store"))][stores - 1]
    ops = collections.Counter(op for op in body[lo:hi] if op.startswith("v_"))
    per_kind = collections.Counter()
    for op, c in ops.items():
        per_kind[kind(op)] += c
    secs = sum(c / rates[k] for k, c in per_kind.items())   # chip-seconds per element-wave
    waves = elements / 64
    return {"kernel": sub, "valu_per_element_wave": sum(ops.values()), "by_kind": dict(per_kind),
            "salu_per_element_wave": sum(1 for op in body[lo:hi] if op.startswith("s_") and op != "s_nop"),
            "s_nop": sum(1 for op in body[lo:hi] if op == "s_nop"),
            "floor_us": round(secs * waves * 1e6, 1),
            "stores": stores,
            "note": "each opcode priced at its kind's saturated chip rate (valu_rate.jsonl, 8 waves/SIMD); "
                    "body = first vector load to the STORES-th vector store"}


# bench.py's kernel legs on the long double every-member fold: 8 sources x
# 32 MiB (2 Mi x87 elements), 8 outputs, each stored when its chain ends
BENCH_LEGS = {
    "rs_shard_n8_longdouble_sum": ("combine_orders_vec<0, x80, 8, 1, 1, true, false>", 2097152, 8),
    "rs_shard_n8_longdouble_prod": ("combine_orders_vec<1, x80, 8, 1, 1, true, false>", 2097152, 8),
}


def main():
    if sys.argv[1] == "--bench-legs":
        print(json.dumps({leg: floor(sys.argv[2], sub, sys.argv[3], n, st)
                          for leg, (sub, n, st) in BENCH_LEGS.items()}))
        return
    obj, sub, rates_path, elements = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    stores = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    print(json.dumps(floor(obj, sub, rates_path, elements, stores)))


if __name__ == "__main__":
    main()
