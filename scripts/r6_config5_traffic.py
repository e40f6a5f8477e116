"""Config 5's HBM traffic per rank step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes over scripts/r6_config5_profile.py (one process per pass):

    python scripts/r6_config5_traffic.py gpurun_out/r6w profiles/config5_traffic.json

Per kernel of the step: the per-launch average of FETCH_SIZE(KiB) * 1024 * 2 +
WRITE_SIZE(KiB) * 1024 (the gfx950 correction of MI355X_MICROARCH.md 'HBM', as
summarize_profile.py); the step's traffic is their sum (one launch each)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import pmc  # noqa: E402

KERNELS = {
    "config5_count_build": "jx_extract_kernel<true, true, 1, false, false, 3, false, 1>",
    "config5_send_probe_one_pass": "jx_extract_kernel<false, true, 2, false, false, 3, false, 3>",
    "config5_emit_build": "jx_extract_kernel<true, true, 2, false, false, 3, false, 2>",
    "config5_ent_build": "jx_ent_build_kernel",
    "config5_ent_part": "jx_ent_part_kernel",
    "config5_part_probe": "jx_part_probe_kernel",
    "config5_ent_first": "jx_ent_first_kernel",
}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    per = {}
    for name, pat in KERNELS.items():
        f = pmc(os.path.join(src, "fetch"), pat)
        w = pmc(os.path.join(src, "write"), pat)
        if "FETCH_SIZE" in f:
            per[name] = f["FETCH_SIZE"] * 1024 * 2 + w.get("WRITE_SIZE", 0.0) * 1024
    out = {"rows_total": 1_000_000_000, "ranks": 8, "rank_file_bytes": 4_000_000_000,
           "hbm_bytes_per_step": sum(per.values()), "per_kernel": per,
           "source": src + " (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE over scripts/r6_config5_profile.py)",
           "correction": "FETCH_SIZE(KiB)*1024*2 + WRITE_SIZE(KiB)*1024 per launch (MI355X_MICROARCH.md HBM)",
           "note": "the users count pass and its emit pass each read the rank's 2.0 GB users share; the orders "
                   "share is read once (one-pass send); the partition pass writes and re-reads the probe entries; "
                   "the receive copy standing in for the xGMI transfer is not a kernel of the step"}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
