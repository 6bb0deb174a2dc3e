#!/usr/bin/env python3
"""ipc_reopen_probe.py -- what this HIP does when an IPC handle is opened again
after its importer closed it (csrc/extmap.c, note 5).

Two processes on one GPU, driven by this script (no GPU in the parent):
  exporter  hipMalloc 4 MiB, fill it, hipIpcGetMemHandle; prints the handle;
            on request re-exports (hipIpcGetMemHandle again, same allocation)
            and prints the new handle; exits when told to.
  importer  runs the sequence below on the exporter's handle(s) and prints
            one JSON line: every step's HIP return code and whether the data
            read through the mapping was the exporter's.
    1 open h1                       (first import)
    2 read through it, close it
    3 open h1 again                 (the re-open of a handle whose only importer closed it)
    4 read, keep it open; open h1 a second time while the first mapping lives
    5 close both
    6 exporter re-exports: h2; same bytes as h1?; open h2, read, close
    7 open h1 once more             (the old handle after a re-export), keep it open
    8 exporter frees the allocation and allocates again (same size), fills it
      with another pattern and exports: h3; same address, same bytes as h1?
    9 read through the mapping kept from step 7; open h3: same address as
      that mapping? reads the new pattern?
   10 close everything; open h1 again (a handle of a freed allocation)
   12 (exporter) 100 more exports of the live allocation: distinct handle
      bytes, and the exporter's open file descriptors before / after
   11 open + read + close h3 CYCLES times (the 3-entry cache of the outside-heap
      stress closes and reopens mappings all the time): first failure, and
      this process's open file descriptors before / after
usage: ipc_reopen_probe.py            -> prints the importer's JSON line
       ipc_reopen_probe.py exporter | importer HEX [HEX2]   (internal)
"""
import ctypes
import json
import os
import subprocess
import sys

SIZE = 4 << 20
PATTERN = 0x5EED0000ABCD1234
PATTERN2 = 0x0DDBA11000000002
CYCLES = 3000


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipGetErrorString.restype = ctypes.c_char_p
    return lib


def err(lib, rc):
    return {"rc": rc, "msg": lib.hipGetErrorString(rc).decode()}


def exporter():
    lib = hip()
    p = ctypes.c_void_p()
    assert lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(SIZE)) == 0
    host = (ctypes.c_uint64 * (SIZE // 8))(*([PATTERN] * (SIZE // 8)))
    assert lib.hipMemcpy(p, host, ctypes.c_size_t(SIZE), 1) == 0
    assert lib.hipDeviceSynchronize() == 0
    for line in sys.stdin:
        cmd = line.strip()
        if cmd == "realloc":
            old = p.value
            old_id = ctypes.c_ulonglong()
            lib.hipPointerGetAttribute(ctypes.byref(old_id), 7, p)  # HIP_POINTER_ATTRIBUTE_BUFFER_ID
            lib.hipFree(p)
            p = ctypes.c_void_p()
            assert lib.hipMalloc(ctypes.byref(p), ctypes.c_size_t(SIZE)) == 0
            host = (ctypes.c_uint64 * (SIZE // 8))(*([PATTERN2] * (SIZE // 8)))
            assert lib.hipMemcpy(p, host, ctypes.c_size_t(SIZE), 1) == 0
            assert lib.hipDeviceSynchronize() == 0
            h = Handle()
            rc = lib.hipIpcGetMemHandle(ctypes.byref(h), p)
            new_id = ctypes.c_ulonglong()
            lib.hipPointerGetAttribute(ctypes.byref(new_id), 7, p)
            print(json.dumps({"rc": rc, "handle": bytes(h).hex() if rc == 0 else None, "same_address": p.value == old,
                              "buffer_id_old_new": [old_id.value, new_id.value]}), flush=True)
        elif cmd == "export":
            h = Handle()
            rc = lib.hipIpcGetMemHandle(ctypes.byref(h), p)
            print(json.dumps({"rc": rc, "handle": bytes(h).hex() if rc == 0 else None}), flush=True)
        elif cmd == "export_many":  # 100 exports of the live allocation: fds and handle bytes
            fd0 = len(os.listdir("/proc/self/fd"))
            seen = set()
            rcs = set()
            for _ in range(100):
                h = Handle()
                rcs.add(lib.hipIpcGetMemHandle(ctypes.byref(h), p))
                seen.add(bytes(h))
            print(json.dumps({"rcs": sorted(rcs), "distinct_handles": len(seen),
                              "fds_before_after": [fd0, len(os.listdir("/proc/self/fd"))]}), flush=True)
        elif cmd == "quit":
            break
    lib.hipFree(p)


def importer(hexes):
    lib = hip()
    out = {}
    h1 = Handle.from_buffer_copy(bytes.fromhex(hexes[0]))

    def op(h):
        p = ctypes.c_void_p()
        rc = lib.hipIpcOpenMemHandle(ctypes.byref(p), h, 1)  # hipIpcMemLazyEnablePeerAccess
        return rc, p

    def read(p, want=PATTERN):
        v = ctypes.c_uint64()
        rc = lib.hipMemcpy(ctypes.byref(v), p, ctypes.c_size_t(8), 2)
        lib.hipGetLastError()
        return rc == 0 and v.value == want

    def value(p):
        v = ctypes.c_uint64()
        rc = lib.hipMemcpy(ctypes.byref(v), p, ctypes.c_size_t(8), 2)
        lib.hipGetLastError()
        return {"rc": rc, "value": hex(v.value) if rc == 0 else None}

    rc, p = op(h1)
    out["1_open"] = err(lib, rc)
    if rc == 0:
        out["2_read_ok"] = read(p)
        out["2_close"] = err(lib, lib.hipIpcCloseMemHandle(p))
    rc, p = op(h1)
    out["3_reopen_after_close"] = err(lib, rc)
    lib.hipGetLastError()
    if rc == 0:
        out["4_read_ok"] = read(p)
        rc2, p2 = op(h1)
        out["4_open_again_while_open"] = err(lib, rc2)
        lib.hipGetLastError()
        if rc2 == 0:
            out["4_second_mapping_same_address"] = p2.value == p.value
            out["5_close_second"] = err(lib, lib.hipIpcCloseMemHandle(p2))
        out["5_close_first"] = err(lib, lib.hipIpcCloseMemHandle(p))
    print(json.dumps(out), flush=True)
    # step 6: the parent hands over h2
    line = sys.stdin.readline()
    h2hex = json.loads(line)["handle"]
    out2 = {"6_same_bytes_as_h1": h2hex == hexes[0]}
    h2 = Handle.from_buffer_copy(bytes.fromhex(h2hex))
    rc, p = op(h2)
    out2["6_open_h2"] = err(lib, rc)
    lib.hipGetLastError()
    if rc == 0:
        out2["6_read_ok"] = read(p)
        out2["6_close"] = err(lib, lib.hipIpcCloseMemHandle(p))
    rc, p7 = op(h1)
    out2["7_open_h1_after_reexport"] = err(lib, rc)
    lib.hipGetLastError()
    if rc == 0:
        out2["7_read_ok"] = read(p7)
    print(json.dumps(out2), flush=True)
    # steps 8-10: the parent hands over the exporter's line after its realloc
    d = json.loads(sys.stdin.readline())
    out3 = {"8_same_address": d["same_address"], "8_same_bytes_as_h1": d["handle"] == hexes[0],
            "8_buffer_id_old_new": d["buffer_id_old_new"]}
    if rc == 0:
        out3["9_old_mapping_reads"] = value(p7)
    h3 = Handle.from_buffer_copy(bytes.fromhex(d["handle"]))
    rc3, p3 = op(h3)
    out3["9_open_h3"] = err(lib, rc3)
    lib.hipGetLastError()
    if rc3 == 0:
        out3["9_h3_same_address_as_old_mapping"] = rc == 0 and p3.value == p7.value
        out3["9_h3_reads"] = value(p3)
        out3["9_h3_reads_new_pattern"] = read(p3, PATTERN2)
        lib.hipIpcCloseMemHandle(p3)
    if rc == 0:
        out3["10_close_old_mapping"] = err(lib, lib.hipIpcCloseMemHandle(p7))
    rc, p = op(h1)
    out3["10_open_h1_after_free"] = err(lib, rc)
    lib.hipGetLastError()
    if rc == 0:
        out3["10_h1_reads"] = value(p)
        lib.hipIpcCloseMemHandle(p)
    fd0 = len(os.listdir("/proc/self/fd"))
    first_fail, fds = None, []
    for i in range(CYCLES):
        rc, p = op(h3)
        if rc != 0:
            first_fail = {"cycle": i, **err(lib, rc)}
            lib.hipGetLastError()
            break
        if not read(p, PATTERN2):
            first_fail = {"cycle": i, "read": "wrong"}
            break
        lib.hipIpcCloseMemHandle(p)
        if i in (0, 9, 99, 999):
            fds.append(len(os.listdir("/proc/self/fd")))
    out3["11_cycles"] = CYCLES
    out3["11_first_failure"] = first_fail
    out3["11_fds_before_after"] = [fd0, len(os.listdir("/proc/self/fd"))]
    out3["11_fds_after_cycles_1_10_100_1000"] = fds
    print(json.dumps(out3), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "exporter":
        return exporter()
    if len(sys.argv) > 1 and sys.argv[1] == "importer":
        return importer(sys.argv[2:])
    me = os.path.abspath(__file__)
    ex = subprocess.Popen([sys.executable, me, "exporter"], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    ex.stdin.write("export\n")
    ex.stdin.flush()
    h1 = json.loads(ex.stdout.readline())
    res = {"export_h1": h1["rc"]}
    im = subprocess.Popen([sys.executable, me, "importer", h1["handle"]], stdin=subprocess.PIPE,
                          stdout=subprocess.PIPE, text=True)
    res.update(json.loads(im.stdout.readline()))
    ex.stdin.write("export\n")
    ex.stdin.flush()
    h2 = ex.stdout.readline()
    res["export_h2"] = json.loads(h2)["rc"]
    im.stdin.write(h2)
    im.stdin.flush()
    res.update(json.loads(im.stdout.readline()))
    ex.stdin.write("realloc\n")
    ex.stdin.flush()
    h3 = ex.stdout.readline()
    res["export_h3"] = json.loads(h3)["rc"]
    im.stdin.write(h3)
    im.stdin.flush()
    res.update(json.loads(im.stdout.readline()))
    im.wait(timeout=120)
    ex.stdin.write("export_many\n")
    ex.stdin.flush()
    res["12_exporter_100_exports"] = json.loads(ex.stdout.readline())
    ex.stdin.write("quit\n")
    ex.stdin.flush()
    ex.wait(timeout=60)
    res["importer_rc"], res["exporter_rc"] = im.returncode, ex.returncode
    print(json.dumps(res))


if __name__ == "__main__":
    main()
