"""Per-phase cycle split of the W&D certified scan (diagnostic build only).

    bash tools/build_variant.sh wdst hnm_recommendation_amd/csrc/widedeep.hip -DWD_STAMPS=1
    HNM_LIB_PATH=$PWD/tools/bin/libhnm_wdst.so python tools/wd_stamps.py

Runs the bench's W&D step (configs[3]: 4,096 users x 105,542 items) twice and reads the
wdc_scan_kernel's s_memtime sums (summed over waves): k loop (layer 2 + the bound MFMAs), the
layer-2 epilogue + layer 3, the per-item bound / top-K / append, and whole tiles.  Shares are
of the tile total; cycles per wave-tile = the sum / (waves x tiles).
"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from hnm_recommendation_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    rd = getattr(lib, "hnm_debug_wd_stamps", None)
    if rd is None:
        raise SystemExit("the loaded library was not built with -DWD_STAMPS=1")
    dev = torch.device("cuda", 0)
    B = 4096
    ret, info, _ = bench.build_workload("widedeep", 0, 1, dev, B)
    users = torch.randint(0, bench.syn.HM_USERS, (B,), device=dev)
    ret["step"](users)
    torch.cuda.synchronize()
    lib.hnm_debug_wd_stamps_reset()
    ret["step"](users)
    torch.cuda.synchronize()
    acc = (C.c_ulonglong * 4)()
    assert rd(acc) == 0
    k, epi, fin, tile = (int(x) for x in acc)
    waves = B // 2
    tiles = -(-bench.syn.HM_ITEMS // 32)
    per = waves * tiles
    print(f"cycles per wave-tile: {tile / per:.0f} (k loop {k / per:.0f}, layer-2 epilogue + "
          f"layer 3 {epi / per:.0f}, bound/top-K/append {fin / per:.0f}, rest "
          f"{(tile - k - epi - fin) / per:.0f})")
    print(f"shares: k loop {k / tile:.3f}, epilogue {epi / tile:.3f}, final {fin / tile:.3f}, "
          f"rest {(tile - k - epi - fin) / tile:.3f}")


if __name__ == "__main__":
    main()
