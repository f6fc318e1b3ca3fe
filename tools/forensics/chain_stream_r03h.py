"""Root cause of the r03h chain parity failure.

Commit add3326 made `csum_chain_stream_kernel` the default for fragment chains; the
next GPU session's C caller (tests/c/test_batch_abi.c at add3326, `test_chains`: 5000
packets of 0-6 fragments of 1-700 B, hint 350) reported 798 wrong results, e.g.
"packet 15 (2 fragments): c2d2 != a085".  This script replays that failure on the CPU:

1. It rebuilds add3326's C caller against host stubs (tools/forensics/stubs.c: hip*
   on host memory, batch entries as no-ops, `rns_csum_chain_dev` dumps its inputs), so
   the caller's RNG draws exactly the inputs the GPU saw (packet 15 has 2 fragments).
2. It runs a lane-level model of the kernel's SOURCE (64 lanes in lockstep, the row
   lookup through the LDS start marks + max-scan, D = 4 rows in flight, pstart/pend
   prefixes, the in-order owner fold of util.rs:112-119) on those inputs:
   0 wrong results -- the algorithm as written is right.
3. It runs the same model with the defect read off the kernel's gfx950 ISA (hipcc,
   ROCm 7.2): in the pipelined lookups for rows k0+5, k0+6, k0+7 the compiler used the
   VGPR holding the pending entry of row k0+4 (`inf[0]`) as the LDS address temporary
   on the divergent path of lanes whose chunk lies past the region's end (fragment
   found, `v >= total`); the ISA marks the whole `inf[]` tuple implicit-def on that
   path.  Those lanes' row-(k0+4) entries become 0 (no bytes, no start/end prefix),
   so the last rows of a 64-fragment sub-block lose chunks.  Result: 399 wrong
   results per call, x 2 flag settings = 798, packet 15 = 0xc2d2, as on the GPU.

Run from the repo root in this container (needs git history and gcc):
    python tools/forensics/chain_stream_r03h.py
Test infrastructure only: nothing here is part of the product or runs on the GPU.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402  (the checker)

D = 4  # rows in flight (kStreamD)


def fold16(w):
    w = int(w)
    while w > 0xffff:
        w = (w & 0xffff) + (w >> 16)
    return w


def model(arena, foff, flen, first, seed, clobber):
    """Lane-level model of add3326's csum_chain_stream_kernel (complemented results)."""
    n = len(first) - 1
    out = np.zeros(n, np.uint32)
    recs = len(arena)
    lanes = np.arange(64)
    for base in range(0, n, 64):
        p = base + lanes
        live = p < n
        f0 = np.where(live, first[np.minimum(p, n)], 0).astype(np.int64)
        f1 = np.where(live, first[np.minimum(p + 1, n)], 0).astype(np.int64)
        acc = np.where(live, seed[np.minimum(p, n - 1)], 0).astype(np.int64)
        sel = f0 < f1
        F0 = f0[sel].min() if sel.any() else 1 << 40
        F1 = f1[sel].max() if sel.any() else 0
        mark = np.full(64, 0xFFFFFFFF, np.int64)
        fb = F0
        while fb < F1:
            f = fb + lanes
            has = f < F1
            fo = np.where(has, foff[np.minimum(f, len(foff) - 1)], 0).astype(np.int64)
            fl = np.where(has, flen[np.minimum(f, len(flen) - 1)], 0).astype(np.int64)
            fs = fo & 15
            nch = np.where(fl > 0, (fs + fl + 15) >> 4, 0)
            vincl = np.cumsum(nch)
            vex = vincl - nch
            total = int(vincl[63])
            nrows = (total + 63) >> 6
            endb = np.where(nch > 0, ((fs + fl - 1) & 15) + 1, 16)
            finfo = [(int(fo[l] & ~15), int(vex[l]), int(fs[l]), int(endb[l]), int(nch[l])) for l in range(64)]
            mark[:] = 0xFFFFFFFF
            active = [0]
            ring = []

            def lookup(k):
                for l in range(64):  # a fragment's first chunk marks its lane in row k
                    if nch[l] and (vex[l] >> 6) == k:
                        mark[vex[l] & 63] = (k << 7) | (l + 1)
                vals = np.where((mark >> 7) == k, mark & 127, 0)
                jj = np.maximum(np.maximum.accumulate(vals), active[0])  # wave_incl_max + carried
                active[0] = int(jj[63])
                if clobber and k >= D + 1 and k % D != 0:  # the ISA defect (module docstring)
                    for l in range(64):
                        if (k << 6) + l >= total and jj[l] != 0:
                            ring[0][l] = None
                info = []
                for l in range(64):
                    v = (k << 6) + l
                    if not (jj[l] != 0 and v < total):
                        info.append(None)
                        continue
                    a0, vx, s0, eb, nc = finfo[jj[l] - 1]
                    rel = v - vx
                    info.append((jj[l] - 1, a0 + rel * 16, s0 if rel == 0 else 0, eb if rel == nc - 1 else 16,
                                 rel == 0, rel == nc - 1))
                return info

            pstart = np.zeros(64, np.int64)
            pend = np.zeros(64, np.int64)
            for j in range(D):
                ring.append(lookup(j))
            carry = 0
            for k0 in range(0, nrows, D):
                for j in range(D):
                    info = ring[j]
                    s = np.zeros(64, np.int64)
                    for l in range(64):
                        if info[l] is None:
                            continue
                        _, addr, lo, hi, _, _ = info[l]
                        ch = arena[addr:addr + 16].astype(np.int64) if addr + 16 <= recs else np.zeros(16, np.int64)
                        ch[:lo] = 0
                        ch[hi:] = 0
                        s[l] = int((ch[0::2] + (ch[1::2] << 8)).sum())
                    ring[j] = lookup(k0 + j + D)
                    inc = np.cumsum(s)
                    for l in range(64):
                        if info[l] is None:
                            continue
                        jl, _, _, _, isf, isl = info[l]
                        if isf:
                            pstart[jl] = carry + inc[l] - s[l]
                        if isl:
                            pend[jl] = carry + inc[l]
                    carry += int(inc[63])
            g = np.zeros(64, np.int64)
            for l in range(64):
                x = fold16((int(pend[l]) - int(pstart[l])) & 0xFFFFFFFF if nch[l] else 0)
                g[l] = x if (fo[l] & 1) else (((x & 0xff) << 8) | (x >> 8))
            for l in range(64):
                for t in range(max(f0[l], fb), min(f1[l], fb + 64)):
                    s_ = (acc[l] & 0xffff) + g[t - fb]
                    acc[l] = (s_ & 0xffff) + (s_ >> 16)
            fb += 64
        for l in range(64):
            if live[l]:
                out[base + l] = (acc[l] & 0xffff) ^ 0xffff
    return out


def dump_inputs(workdir):
    caller = os.path.join(workdir, "caller.c")
    hdr = os.path.join(workdir, "rns_checksum.h")
    for path, spec in ((caller, "add3326:tests/c/test_batch_abi.c"), (hdr, "add3326:include/rns_checksum.h")):
        with open(path, "wb") as f:
            f.write(subprocess.check_output(["git", "-C", ROOT, "show", spec]))
    hc = os.path.join(workdir, "hc.o")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", workdir, "-c",
                           os.path.join(ROOT, "rustnetworkstack_amd/csrc/host_checksum.cpp"), "-o", hc])
    exe = os.path.join(workdir, "replay")
    subprocess.check_call(["gcc", "-std=gnu11", "-O1", "-w", "-D__HIP_PLATFORM_AMD__", "-I", workdir,
                           "-I/opt/rocm/include", caller, os.path.join(ROOT, "tools/forensics/stubs.c"),
                           os.path.join(ROOT, "oracle/csum_oracle.c"), hc, "-lstdc++", "-lpthread", "-o", exe])
    subprocess.run([exe], cwd=workdir, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    raw = open(os.path.join(workdir, "chain_inputs.bin"), "rb").read()
    nbytes, nf, npk = [int(x) for x in np.frombuffer(raw[:24], np.uint64)]
    o = 24
    arena = np.frombuffer(raw[o:o + nbytes], np.uint8)
    o += nbytes
    foff = np.frombuffer(raw[o:o + 8 * nf], np.uint64).astype(np.int64)
    o += 8 * nf
    flen = np.frombuffer(raw[o:o + 4 * nf], np.uint32).astype(np.int64)
    o += 4 * nf
    first = np.frombuffer(raw[o:o + 4 * (npk + 1)], np.uint32).astype(np.int64)
    o += 4 * (npk + 1)
    seed = np.frombuffer(raw[o:o + 2 * npk], np.uint16).astype(np.int64)
    return arena, foff, flen, first, seed


def main():
    with tempfile.TemporaryDirectory() as wd:
        arena, foff, flen, first, seed = dump_inputs(wd)
    npk = len(first) - 1
    blob = bytes(arena)
    want = []
    for i in range(npk):
        s = int(seed[i])
        for f in range(first[i], first[i + 1]):
            s = O.ones_comp_py(s, blob[foff[f]:foff[f] + flen[f]])
        want.append(s ^ 0xffff)
    print(f"inputs: {npk} packets, {len(foff)} fragments; packet 15 has {first[16] - first[15]} fragments, "
          f"oracle {want[15]:04x}")
    for clobber in (False, True):
        got = model(arena, foff, flen, first, seed, clobber)
        bad = sum(int(got[i]) != want[i] for i in range(npk))
        print(f"{'source as written' if not clobber else 'with the ISA clobber':22s}: {bad} wrong of {npk} "
              f"(x2 flag settings = {2 * bad}); packet 15 -> {int(got[15]):04x}")


if __name__ == "__main__":
    main()
