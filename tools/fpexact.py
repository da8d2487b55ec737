"""Full bit-exactness sweeps of the kernels' short correctly rounded f32 sequences
(rrte_hip_fpcheck): sqrt and 1/x over all 2^32 inputs, the constant-divisor division step over
all 2^46 significand pairs.  usage: python tools/fpexact.py [sqrt|rcp|div ...]  (MI355X)"""
import ctypes as C
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from rrte_amd import abi  # noqa: E402

KINDS = {"sqrt": (abi.FPCHECK_SQRT, 1 << 32), "rcp": (abi.FPCHECK_RCP, 1 << 32), "div": (abi.FPCHECK_DIV, 1 << 23),
         "sqrt_hw": (abi.FPCHECK_SQRT_HW, 1 << 32), "sqrt_bf": (abi.FPCHECK_SQRT_BF, 1 << 32),
         "gamma": (abi.FPCHECK_GAMMA_U8, 1 << 32)}  # control: the bare 1-ulp v_sqrt_f32


def main():
    lib = abi.load()
    res = {}
    for name in sys.argv[1:] or ["sqrt", "rcp", "div", "sqrt_hw"]:
        kind, hi = KINDS[name]
        t0, bad, step = time.time(), 0, hi // 16
        for lo in range(0, hi, step):  # progress line per sixteenth
            out = C.c_uint64(0)
            st = lib.rrte_hip_fpcheck(0, kind, lo, lo + step, C.byref(out))
            if st != 0:
                raise SystemExit(f"{name}: status {abi.STATUS_NAMES.get(st, st)}")
            bad += out.value
            print(f"{name}: {lo + step}/{hi} mismatches so far {bad}", file=sys.stderr, flush=True)
        res[name] = {"cases": hi if name != "div" else hi << 23, "mismatches": bad, "seconds": round(time.time() - t0, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
