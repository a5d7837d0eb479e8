"""Lists, per kernel of a HIP source, the barriers and the `s_waitcnt vmcnt(0)`
sites of its gfx950 assembly (line numbers in the kernel body).  A full wait
right after a conditional load, or at the join of a uniform branch, makes
the wave wait for EVERY load in flight, including prefetches meant to land
later (round 6: the n <= 32 attention kernels' softmax waited for the whole
graph's xs that way).  Usage: python tools/waitscan.py SRC.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
asm = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                      "-Iinclude", "--cuda-device-only", "-S", src, "-o", "/dev/stdout"],
                     capture_output=True, text=True).stdout
for m in re.finditer(r"^(_Z\S+):", asm, re.M):
    name = m.group(1)
    if not rx.search(name):
        continue
    body = [x.strip() for x in asm[m.end():asm.find(".Lfunc_end", m.end())].split("\n")]
    bars = [i for i, x in enumerate(body) if x.startswith("s_barrier")]
    full = [i for i, x in enumerate(body) if x.startswith("s_waitcnt") and "vmcnt(0)" in x]
    print(f"{name[:70]:70s} lines {len(body):6d} barriers {bars[:6]} vmcnt(0) x{len(full)} {full[:8]}")
