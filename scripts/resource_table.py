"""Per-kernel resource table (VGPRs, AGPRs, SGPRs, scratch, LDS, occupancy) of
the libhq kernel sources, from hipcc's kernel-resource-usage remarks.

    python scripts/resource_table.py [FILTER] [-D...]
"""
import re
import subprocess
import sys

SRC = ["hq_search.hip", "hq_assign.hip", "hq_cost.hip", "hq_setup.hip", "hq_wide.hip", "hq_lists16.hip"]
CSRC = "hybridquantization_amd/csrc"


def main():
    filt = next((a for a in sys.argv[1:] if not a.startswith("-")), "")
    extra = [a for a in sys.argv[1:] if a.startswith("-")]
    for f in SRC:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
               "-munsafe-fp-atomics", "-Rpass-analysis=kernel-resource-usage", "-c", f"{CSRC}/{f}",
               "-o", "/dev/null", *extra]
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
        cur = None
        for line in out.splitlines():
            m = re.search(r"remark: (?:\S+: )?\s*(Function Name|Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|"
                          r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (.*?) \[-Rpass", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k in ("Function Name", "Name"):
                cur = {"name": v}
            elif cur is not None:
                cur[k] = v
                if k.startswith("LDS"):
                    name = subprocess.run(["c++filt", cur["name"]], capture_output=True, text=True).stdout.strip()
                    if filt in name:
                        print(f"{name[:70]:70s} V{cur.get('VGPRs', '?'):>4} A{cur.get('AGPRs', '?'):>3} "
                              f"S{cur.get('TotalSGPRs', '?'):>4} scr{cur.get('ScratchSize [bytes/lane]', '?'):>4} "
                              f"occ{cur.get('Occupancy [waves/SIMD]', '?'):>2} lds{v:>6}")
                    cur = None


if __name__ == "__main__":
    main()
