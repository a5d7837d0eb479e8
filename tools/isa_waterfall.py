"""(1) Reports kernels whose buffer loads / stores sit in waterfall loops (a
resource descriptor or soffset the compiler cannot prove wave-uniform is
made uniform lane by lane: v_readfirstlane + s_and_saveexec around the
memory instruction, one loop per instruction).  (2) Reports a v_readfirstlane
writing an SGPR that a buffer / global instruction reads within 5 wait states
(the VALU-writes-SGPR -> VMEM-reads-it hazard; an inline-asm readfirstlane does
not get the compiler's wait states, and round 5 faulted a GPU on exactly
that: a stale buffer descriptor).  Usage:
    python tools/isa_waterfall.py spotv2net_amd/csrc/*.hip"""
import re
import subprocess
import sys

nk = nwf = nhz = 0
for src in sys.argv[1:]:
    asm = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                          "-Iinclude", "--cuda-device-only", "-S", src, "-o", "/dev/stdout"],
                         capture_output=True, text=True).stdout
    for m in re.finditer(r"^(_Z\S+):\s*;?.*\n", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        body = asm[m.end():end]
        wf = 0
        nk += 1
        for h in re.finditer(r"; =>This Inner Loop Header", body):
            seg = body[h.start():body.find("s_cbranch_execnz", h.start()) + 1].split("\n")[1:]
            # the waterfall shape: readfirstlanes first, then a compare, the
            # exec mask, one buffer instruction, the exec flip, the back edge
            wf += bool(len(seg) < 24 and seg and "v_readfirstlane" in seg[0]
                   and any("s_and_saveexec" in x for x in seg)
                   and any("buffer_" in x for x in seg))
        if wf:
            nwf += 1
            print(f"{src.split('/')[-1]}: {m.group(1)[:100]} waterfall buffer ops: {wf}")
        lines = body.split("\n")
        for k, ln in enumerate(lines):
            r = re.search(r"v_readfirstlane_b32 s(\d+), v", ln)
            if not r:
                continue
            reg, ws = int(r.group(1)), 0
            for l2 in lines[k + 1:k + 30]:
                tt = l2.strip()
                if not tt or tt[0] in ";.":
                    continue
                nop = re.match(r"s_nop (\d+)", tt)
                ws += int(nop.group(1)) + 1 if nop else 1
                if ws > 5:
                    break
                if re.search(r"(buffer_|global_)", tt) and any(
                        int(a) <= reg <= int(b) for a, b in re.findall(r"s\[(\d+):(\d+)\]", tt)):
                    nhz += 1
                    print(f"{src.split('/')[-1]}: {m.group(1)[:100]} HAZARD: {ln.strip()} -> {tt}")
print(f"{nk} kernels in {len(sys.argv) - 1} sources: {nwf} with waterfall buffer ops, "
      f"{nhz} readfirstlane -> VMEM hazards")
