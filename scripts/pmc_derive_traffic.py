#!/usr/bin/env python3
"""Per-launch HBM traffic of the derive-mode launches from a per-kernel PMC
summary (scripts/pmc_by_kernel.py over `exp_derive.py --reps 0`: one levels
launch over all V roots and one derive launch per class), written into
profiles/<round>/pmc_traffic.json under the keys bench.py reads:
derive_levels (lv_init / level / settle / rows, or the 64-root msbfs ones, + the
state memsets), derive_cap8 (nh_derive16_kernel<1>), derive_cap96
(nh_derive16_kernel<3>), derive_cap1792 (nh_derive_wide_kernel).
hbm bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB (MI355X_MICROARCH.md: FETCH_SIZE
x 2 on gfx950). Usage: pmc_derive_traffic.py PMC_JSON V N_CAP8 N_CAP96 N_CAP1792 OUT_JSON"""
import json
import os
import sys


def main():
    pmc, V, n8, n96, nw, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), \
        int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
    d = json.load(open(pmc))
    groups = {
        "derive_levels": (V, [k for k in d if ("<-1>" in k or "levrows" in k or "fillBuffer" in k
                                              or k.startswith("lv_"))]),
        "derive_cap8": (n8, [k for k in d if k == "nh_derive16_kernel<1>"]),
        "derive_cap96": (n96, [k for k in d if k == "nh_derive16_kernel<3>"]),
        "derive_cap1792": (nw, [k for k in d if k == "nh_derive_wide_kernel"]),
    }
    res = json.load(open(out)) if os.path.exists(out) else {}
    for key, (roots, ks) in groups.items():
        if not ks:
            continue
        f = sum(d[k].get("FETCH_SIZE", 0.0) for k in ks)
        w = sum(d[k].get("WRITE_SIZE", 0.0) for k in ks)
        res[key] = {"roots_per_launch": roots, "launches": 1, "kernels": ks,
                    "fetch_size_kib_per_launch": f, "write_size_kib_per_launch": w,
                    "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
                    "hbm_bytes_per_root": int(round((2 * f + w) * 1024 / roots)),
                    "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over "
                              "scripts/exp_derive.py --reps 0 (scripts/pmc_by_kernel.py)"}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
