#!/usr/bin/env python3
"""Emit the 44 reduction prototypes for include/shmem.h and include/pshmem.h.

The type/op matrix follows reference src/reduce/reduce-op.c:405-448 and the
prototype order of src/shmem.h:1507-1743. Run once; output is pasted into the
headers (kept as a tool so the matrix has one source of truth).
"""
TYPES = {
    "short": "short", "int": "int", "long": "long", "longlong": "long long",
    "float": "float", "double": "double", "longdouble": "long double",
    "complexf": "COMPLEXIFY (float)", "complexd": "COMPLEXIFY (double)",
}
MATRIX = [
    ("sum", ["short", "int", "long", "longlong", "float", "double", "longdouble", "complexf", "complexd"]),
    ("prod", ["short", "int", "long", "longlong", "float", "double", "longdouble", "complexf", "complexd"]),
    ("and", ["short", "int", "long", "longlong"]),
    ("or", ["short", "int", "long", "longlong"]),
    ("xor", ["short", "int", "long", "longlong"]),
    ("max", ["short", "int", "long", "longlong", "float", "double", "longdouble"]),
    ("min", ["short", "int", "long", "longlong", "float", "double", "longdouble"]),
]


def protos(prefix):
    out = []
    for op, names in MATRIX:
        for n in names:
            t = TYPES[n]
            out.append(f"void {prefix}_{n}_{op}_to_all ({t} *target, {t} *source,\n"
                       f"        int nreduce, int PE_start, int logPE_stride, int PE_size,\n"
                       f"        {t} *pWrk, long *pSync);")
    return "\n".join(out)


def stream_protos():
    """shmemx.h: the stream-ordered variants (same arguments, plus the stream)."""
    out = []
    for op, names in MATRIX:
        for n in names:
            t = TYPES[n]
            out.append(f"void shmemx_{n}_{op}_to_all_on_stream ({t} *target, {t} *source,\n"
                       f"        int nreduce, int PE_start, int logPE_stride, int PE_size,\n"
                       f"        {t} *pWrk, long *pSync, void *stream);")
    return "\n".join(out)


if __name__ == "__main__":
    import sys
    arg = sys.argv[1] if len(sys.argv) > 1 else "shmem"
    print(stream_protos() if arg == "stream" else protos(arg))
