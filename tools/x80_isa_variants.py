#!/usr/bin/env python3
"""x80_isa_variants.py -- code-object variants of x80_lane_probe's `general`
kernels, for the round-2 x87 nondeterminism.

Takes the probe's own device assembly (hipcc --cuda-device-only -S), and for the
two general kernels (fold3<0,0> add, fold3<1,0> mul) inserts `s_nop N` after the
instructions a rule selects, then assembles and links each variant into a code
object the probe loads (`x80_lane_probe ... <code object>`). The unmodified
variant `orig` must reproduce the built-in kernel's behaviour (its disassembly is
the compiler's, instruction for instruction); a rule whose nops remove the errors
names the instruction class whose result is consumed too early.

usage: x80_isa_variants.py <device.s> <out dir> [rule ...]
"""
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
KERNELS = ("_Z5fold3ILi0ELi0EEvPK3x80S2_S2_PS0_Pjm", "_Z5fold3ILi1ELi0EEvPK3x80S2_S2_PS0_Pjm")

INSN = re.compile(r"^\s+([sv]_[a-z0-9_]+|global_[a-z0-9_]+|buffer_[a-z0-9_]+)\b(.*)$")
SDST_VOP3B = ("v_add_co_u32", "v_sub_co_u32", "v_subrev_co_u32", "v_addc_co_u32", "v_subb_co_u32",
              "v_subbrev_co_u32", "v_mad_u64_u32", "v_mad_i64_i32", "v_div_scale_f32", "v_div_scale_f64")
SGPR = r"(vcc|exec|s\d+|s\[\d+:\d+\])"
NO_NOP_AFTER = ("s_endpgm", "s_branch", "s_cbranch", "s_setpc", "s_nop", "s_waitcnt")


def operands(rest):
    rest = rest.split(";")[0].split("//")[0]
    return [o.strip() for o in rest.split(",") if o.strip()]


def valu_writes_sgpr(op, ops):
    if not op.startswith("v_") or not ops:
        return False
    if re.fullmatch(SGPR, ops[0]):  # v_cmp_*_e64 s[..], v_cmp_*_e32 vcc, v_readfirstlane sN
        return True
    return op.split("_e")[0] in SDST_VOP3B and len(ops) > 1 and re.fullmatch(SGPR, ops[1]) is not None


def base(op):  # opcode without its encoding suffix (_e32 / _e64 / _sdwa / _dpp)
    return re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)


def is_64bit_valu(op, ops):  # 64-bit operands: shifts, compares, v_mad_u64_u32, v_lshl_add_u64, moves
    return op.startswith("v_") and "64" in base(op)


def cmp64(op, ops):
    return valu_writes_sgpr(op, ops) and op.startswith("v_cmp") and "64" in base(op)


def cmp_narrow(op, ops):
    return valu_writes_sgpr(op, ops) and op.startswith("v_cmp") and "64" not in base(op)


def carry(op, ops):
    return valu_writes_sgpr(op, ops) and not op.startswith("v_cmp")


RULES = {
    "orig": lambda op, ops: False,
    "valu_sgpr": valu_writes_sgpr,                      # VALU result in an SGPR / VCC (compare masks, carries)
    "salu": lambda op, ops: op.startswith("s_") and not op.startswith(NO_NOP_AFTER),
    "valu64": is_64bit_valu,                            # 64-bit shifts, compares, multiplies
    "valu": lambda op, ops: op.startswith("v_"),        # every VALU instruction
    "vmem": lambda op, ops: op.startswith(("global_", "buffer_")),
    "all": lambda op, ops: not op.startswith(NO_NOP_AFTER),
    "cmp64": cmp64,                                     # 64-bit compares into an SGPR mask / VCC
    "cmp_narrow": cmp_narrow,                           # 16/32-bit compares into an SGPR mask / VCC
    "carry": carry,                                     # carry/borrow outs (v_sub_co, v_subb_co, v_mad_u64_u32)
}


def kernel_lengths(lines):
    """instructions per target kernel (for the slice rules)"""
    n, inside, cur = {}, False, None
    for ln in lines:
        for k in KERNELS:
            if ln.startswith(k + ":"):
                inside, cur = True, k
                n[k] = 0
        if inside and (ln.startswith(".Lfunc_end") or "s_endpgm" in ln):
            inside = False
        elif inside and INSN.match(ln):
            n[cur] += 1
    return n


def transform(lines, rule, nops):
    """rule: a RULES name, or slice/I/K: every instruction in the I-th of K equal slices of each
    target kernel (by instruction count)"""
    out, inside, sites, idx, cur = [], False, 0, 0, None
    sl = None
    if rule.startswith("slice/"):
        _, i, k = rule.split("/")
        sl, lens = (int(i), int(k)), kernel_lengths(lines)
    for ln in lines:
        out.append(ln)
        if any(ln.startswith(k + ":") for k in KERNELS):
            inside, idx = True, 0
            cur = next(k for k in KERNELS if ln.startswith(k + ":"))
            continue
        if inside and (ln.startswith(".Lfunc_end") or "s_endpgm" in ln):
            inside = False
            continue
        if not inside:
            continue
        m = INSN.match(ln)
        if m is None:
            continue
        op, ops = m.group(1), operands(m.group(2))
        idx += 1
        if sl is not None:
            n = lens[cur]
            hit = sl[0] * n // sl[1] <= idx - 1 < (sl[0] + 1) * n // sl[1] and not op.startswith(NO_NOP_AFTER)
        else:
            hit = RULES[rule](op, ops)
        if hit:
            out.append("\ts_nop %d\n" % nops)
            sites += 1
    return out, sites


def main():
    src, outdir = sys.argv[1], sys.argv[2]
    rules = sys.argv[3:] or list(RULES)
    os.makedirs(outdir, exist_ok=True)
    lines = open(src).readlines()
    for spec in rules:
        rule, _, n = spec.partition(":")
        nops = int(n) if n else 4
        var, sites = transform(lines, rule, nops)
        base = os.path.join(outdir, "general_%s%s" % (rule.replace("/", "-"), "_%d" % nops if n else ""))
        open(base + ".s", "w").writelines(var)
        subprocess.check_call([LLVM + "/clang", "-x", "assembler", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950",
                               "-c", base + ".s", "-o", base + ".o"])
        subprocess.check_call([LLVM + "/ld.lld", "-shared", base + ".o", "-o", base + ".hsaco"])
        os.remove(base + ".o")
        print("%-40s %4d nop sites" % (base + ".hsaco", sites))


if __name__ == "__main__":
    main()
