"""A/B of library builds on the same box: device time of rns_csum_batch_dev_off32
(compact descriptors, the pick_shape default kernel) for c3 and IMIX, calling the
given .so directly through ctypes (an older build need not export today's symbols).

    python tools/probe_lib_ab.py <lib.so> [label]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    path, label = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1]))
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.rns_csum_batch_dev_off32
    f.restype = ctypes.c_int
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    f.argtypes = [vp, u64, vp, vp, vp, vp, u32, u32, u32, vp, vp]
    from rustnetworkstack_amd.workloads import make_layout, splitmix64
    dev = torch.device("cuda:0")
    res = {"label": label}
    for name in ("c5_imix", "c3_1500B", "c5_imix"):
        lay = make_layout(name)
        arena = torch.empty(lay.arena_bytes + 16, dtype=torch.uint8, device=dev)
        # fill with torch on the device (no dependence on the library under test)
        g = torch.Generator(device=dev).manual_seed(lay.data_seed & 0x7FFFFFFF)
        arena.copy_(torch.randint(0, 256, arena.shape, dtype=torch.uint8, device=dev, generator=g))
        off = torch.from_numpy(lay.off.astype(np.uint32).view(np.int32)).to(dev)
        ln = torch.from_numpy(lay.length.view(np.int32)).to(dev)
        sd = torch.from_numpy(lay.seed.view(np.int16)).to(dev)
        out = torch.empty(lay.n, dtype=torch.int16, device=dev)
        args = (arena.data_ptr(), arena.numel(), off.data_ptr(), ln.data_ptr(), sd.data_ptr(), out.data_ptr(),
                lay.n, 1, int(round(lay.mean_len)), None, None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            assert f(*args) == 0
        ts = []
        for _ in range(5):
            e0.record()
            for _ in range(20):
                f(*args)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        key = name if name not in res else name + "_again"
        res[key] = round(sorted(ts)[2], 1)
        res[key + "_checksum_of_results"] = int(out.to(torch.int64).sum().item())
        del arena, off, ln, sd, out
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
