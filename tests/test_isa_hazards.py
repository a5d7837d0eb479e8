"""Machine-code guard for the round-5 GPU fault ("No waterfall
loops around buffer instructions"), run over the gfx950 code objects of the
BUILT library, not over a recompile of the sources:

1. no buffer load / store inside a waterfall loop (v_readfirstlane +
   s_and_saveexec + the memory instruction + s_cbranch_execnz back to the
   readfirstlane: a descriptor or soffset the compiler could not prove
   wave-uniform, made uniform lane by lane, one loop per instruction);
2. no v_readfirstlane writing an SGPR that a buffer / global instruction
   reads within 5 wait states (VALU writes SGPR -> VMEM reads it; the
   hardware needs wait states there, the compiler inserts them only for code
   it generated itself, and an inline-asm readfirstlane that skipped them
   made a buffer load read a stale descriptor: round 5, one faulted GPU run).

The code objects are taken out of the library's offload bundles
(``__CLANG_OFFLOAD_BUNDLE__`` entries for ``amdgcn-amd-amdhsa--gfx950``) and
disassembled with the ROCm llvm-objdump.  ``libsv2n_check.so`` (``make
CHECK=1``) is scanned too when it has been built."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WAIT_STATES = 5


def code_objects(path):
    """The gfx950 code objects (ELF bytes) bundled into a host shared library."""
    data = open(path, "rb").read()
    out = []
    i = data.find(MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", data, i + len(MAGIC))
        p = i + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                out.append(data[i + off:i + off + size])
        i = data.find(MAGIC, i + len(MAGIC))
    return out


_INSN = re.compile(r"^\s+([a-z_0-9]+)(.*?)//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^([0-9a-f]+) <(\S+)>:")
_TARGET = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")


def parse(disasm):
    """{kernel: [(address, mnemonic, operands)]} of one disassembly."""
    funcs, cur, bases = {}, None, {}
    for ln in disasm.splitlines():
        f = _FUNC.match(ln)
        if f:
            cur = f.group(2)
            bases[cur] = int(f.group(1), 16)
            funcs[cur] = []
            continue
        m = _INSN.match(ln)
        if m and cur is not None:
            funcs[cur].append((int(m.group(3), 16), m.group(1), m.group(2)))
    return funcs, bases


def scan(funcs, bases):
    """(waterfall findings, hazard findings) as lists of strings."""
    waterfalls, hazards = [], []
    for name, ins in funcs.items():
        addr_idx = {a: k for k, (a, _, _) in enumerate(ins)}
        for k, (a, mn, ops) in enumerate(ins):
            if mn == "s_cbranch_execnz":
                t = _TARGET.search(ops)
                if not t or t.group(1) != name:
                    continue
                j = addr_idx.get(bases[name] + int(t.group(2), 16))
                if j is None or j > k or k - j >= 24:
                    continue
                seg = ins[j:k + 1]
                if seg[0][1].startswith("v_readfirstlane") and \
                        any(s[1].startswith("s_and_saveexec") for s in seg) and \
                        any(s[1].startswith("buffer_") for s in seg):
                    waterfalls.append(f"{name[:90]} @0x{a:x}")
            r = re.match(r"v_readfirstlane_b32$", mn) and re.match(r"\s*s(\d+),", ops)
            if not r:
                continue
            reg, ws = int(r.group(1)), 0
            for _, mn2, ops2 in ins[k + 1:k + 1 + 2 * WAIT_STATES]:
                nop = re.match(r"s_nop$", mn2) and re.match(r"\s*(\d+)", ops2)
                ws += int(nop.group(1)) + 1 if nop else 1
                if ws > WAIT_STATES:
                    break
                if mn2.startswith(("buffer_", "global_")) and any(
                        int(lo) <= reg <= int(hi)
                        for lo, hi in re.findall(r"s\[(\d+):(\d+)\]", ops2)):
                    hazards.append(f"{name[:90]} @0x{a:x}: s{reg} -> {mn2}{ops2.rstrip()}")
    return waterfalls, hazards


def _libs():
    libs = [os.path.join(ROOT, "spotv2net_amd", "libsv2n.so")]
    chk = os.path.join(ROOT, "spotv2net_amd", "libsv2n_check.so")
    return libs + ([chk] if os.path.exists(chk) else [])


@pytest.mark.parametrize("lib", _libs(), ids=os.path.basename)
def test_built_library_has_no_waterfall_or_sgpr_hazard(lib):
    if not os.path.exists(OBJDUMP):
        pytest.skip("ROCm llvm-objdump not installed")
    assert os.path.exists(lib), f"{lib} not built (make)"
    cos = code_objects(lib)
    assert cos, "no gfx950 code object in the library"
    nk, wf, hz = 0, [], []
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(cos):
            p = os.path.join(d, f"co{i}.o")
            with open(p, "wb") as f:
                f.write(co)
            dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", p], check=True,
                                 capture_output=True, text=True).stdout
            funcs, bases = parse(dis)
            nk += len(funcs)
            w, h = scan(funcs, bases)
            wf += w
            hz += h
    assert nk > 100, f"only {nk} kernels disassembled"
    assert not wf, "waterfall loops around buffer instructions:\n" + "\n".join(wf[:20])
    assert not hz, "v_readfirstlane -> VMEM SGPR hazards:\n" + "\n".join(hz[:20])


def test_scanner_flags_the_faulting_patterns():
    """The scanner itself, on hand-written disassembly in llvm-objdump's
    format: the round-5 hazard (readfirstlane into a descriptor SGPR read by
    the next buffer load) and a waterfall loop are flagged; the same code
    with the wait states the compiler inserts is not."""
    hdr = "0000000000001000 <k>:\n"

    def ins(a, text):
        return f"\t{text:<58}// {a:012X}: 00000000\n"

    bad = hdr + ins(0x1000, "v_readfirstlane_b32 s8, v1") + \
        ins(0x1004, "buffer_load_dword v2, v3, s[8:11], 0 offen")
    ok = hdr + ins(0x1000, "v_readfirstlane_b32 s8, v1") + ins(0x1004, "s_nop 4") + \
        ins(0x1008, "buffer_load_dword v2, v3, s[8:11], 0 offen")
    loop = hdr + ins(0x1000, "v_readfirstlane_b32 s4, v2") + \
        ins(0x1004, "v_cmp_eq_u32_e32 vcc, s4, v2") + \
        ins(0x1008, "s_and_saveexec_b64 s[6:7], vcc") + ins(0x100c, "s_nop 4") + \
        ins(0x1010, "buffer_load_dword v5, v6, s[8:11], s4 offen") + \
        ins(0x1014, "s_xor_b64 exec, exec, s[6:7]") + \
        ins(0x1018, "s_cbranch_execnz 65529 <k+0x0>")
    assert len(scan(*parse(bad))[1]) == 1
    assert scan(*parse(ok)) == ([], [])
    assert len(scan(*parse(loop))[0]) == 1
