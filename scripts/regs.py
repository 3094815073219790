"""Per-kernel register use of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage), as a table.

    python scripts/regs.py csrc/mnist_cnn.hip [extra hipcc flags ...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed-learning-contributivity_amd")
FILE_FLAGS = {"mnist_cnn.hip": ["-fno-slp-vectorize"], "mnist_wgrad.hip": ["-fno-slp-vectorize"]}


def main():
    src = sys.argv[1]
    if not os.path.exists(src):
        src = os.path.join(PKG, src)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(PKG, "csrc"), "-munsafe-fp-atomics", "-c", src, "-o", "/tmp/_regs.o",
           "-Rpass-analysis=kernel-resource-usage"] + FILE_FLAGS.get(os.path.basename(src), []) + sys.argv[2:]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr)
        sys.exit(1)
    cur = None
    rows = {}
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?)(?: \[-Rpass)", line)
        if not m:
            continue
        txt = m.group(1)
        if txt.startswith("Function Name:"):
            cur = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", txt.split(":", 1)[1].strip())
            cur = re.split(r"E[PKiflSTI]", cur)[0] if "E" in cur else cur
            rows[cur] = {}
        elif cur and ":" in txt:
            k, v = txt.split(":", 1)
            rows[cur][k.strip()] = v.strip()
    keys = ["VGPRs", "AGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
    print("%-40s %6s %6s %6s %8s %4s %8s" % ("kernel", "VGPR", "AGPR", "spill", "scratch", "occ", "LDS"))
    for name, d in rows.items():
        print("%-40s %6s %6s %6s %8s %4s %8s" % ((name[:40],) + tuple(d.get(k, "-") for k in keys)))


if __name__ == "__main__":
    main()
