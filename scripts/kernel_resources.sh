# per-kernel resources of the gfx950 build of one source (VGPRs, AGPRs, scratch, spills,
# occupancy): hipcc -Rpass-analysis=kernel-resource-usage, summarized one line per kernel
#   bash scripts/kernel_resources.sh fast.hip [extra hipcc flags] > profiles/rN_kernel_resources.txt
set -e
cd "$(dirname "$0")/../cq_amd/csrc"
src=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include "$@" \
    -Rpass-analysis=kernel-resource-usage -c "$src" -o /tmp/kr_$$.o 2> /tmp/kr_$$.txt
python3 - /tmp/kr_$$.txt <<'PY'
import re, sys
cur, out = None, {}
for ln in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1); out[cur] = {}; continue
    m = re.search(r"remark: ([^:]+?): (\d+)\s*$", ln.split("kernel-resource-usage")[0] + ln) if False else None
    for key, tag in (("VGPRs:", "V"), ("AGPRs:", "A"), ("ScratchSize [bytes/lane]:", "scr"), ("SGPRs Spill:", "sS"),
                     ("VGPRs Spill:", "vS"), ("Occupancy [waves/SIMD]:", "occ"), ("SGPRs:", "S"), ("LDS Size [bytes/block]:", "lds")):
        if cur and (" " + key) in ln:
            out[cur][tag] = ln.rsplit(key, 1)[1].split("[")[0].strip()
import subprocess
names = list(out)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    r = out[n]
    print(f"{d[:100]:100s} V={r.get('V')} A={r.get('A')} S={r.get('S')} scr={r.get('scr')} sS={r.get('sS')} vS={r.get('vS')} occ={r.get('occ')}")
PY
rm -f /tmp/kr_$$.o /tmp/kr_$$.txt
