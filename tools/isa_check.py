#!/usr/bin/env python3
"""Build-time check of the MTD kernel's hand-counted LDS-DMA wait.

mtd_tile (radar-signal-process_amd/csrc/rsp_kernels.hip, the kMtdDma path) issues the tile's
`buffer_load_dwordx4 ... lds` pieces, then the range job's Hook::kLoads gathers, then an asm
`s_waitcnt vmcnt(Hook::kLoads)` and an `s_barrier`, after which every wave reads the tile from
LDS.  vmcnt counts vector-memory operations in issue order, so the asm wait covers the DMA
pieces only if exactly kLoads VMEM instructions issue between the last piece and the wait.  The
compiler cannot see inside the asm, so nothing at build time enforced that; this script reads
the shipped code object and checks it for every mtd_kernel instance that uses LDS-DMA:

  * between the last DMA piece and the first s_barrier after it there is no branch;
  * the first `s_waitcnt vmcnt(N)` after the last piece that covers it (N <= the VMEM
    instructions issued since the piece) comes before that barrier, and N equals that count
    (an asm count edited up leaves the DMA uncovered at the barrier; edited down, it over-waits
    and drains the gathers: both fail);
  * that count is the hook's kLoads (17 range-job gathers for JOB kernels, 0 otherwise), i.e.
    no gather was hoisted above the DMA and none was dropped or merged.

    python tools/isa_check.py [lib/librsp.so]     exit status 0 = all instances hold
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "radar-signal-process_amd", "lib", "librsp.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
K_JOB_LOADS = 17      # RangeJob57::kLoads (NX: the cells of executeCFAR's fixCells test)
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else name


def disassemble(lib=LIB):
    """gfx950 disassembly of every device code object in the library's .hip_fatbin."""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.check_call([_tool("llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, lib, os.path.join(d, "x")])
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        text = []
        for i, s in enumerate(starts):
            part = os.path.join(d, "b%d.bin" % i)
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, "b%d.co" % i)
            r = subprocess.run([_tool("clang-offload-bundler"), "--type=o", "--targets=" + TARGET, "--input=" + part,
                                "--output=" + co, "--unbundle"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            text.append(subprocess.run([_tool("llvm-objdump"), "-d", "--mcpu=gfx950", co], capture_output=True,
                                       text=True, check=True).stdout)
        return "\n".join(text)


def functions(asm):
    """{mangled name: [instruction lines]} of the disassembly."""
    out, cur = {}, None
    for ln in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:\s*$", ln)
        if m:
            cur = out.setdefault(m.group(1), [])
            continue
        if cur is not None:
            s = ln.strip()
            if s and not s.startswith(";"):
                cur.append(s.split("//")[0].strip())
    return out


_VMEM = re.compile(r"^(buffer|global|flat|scratch)_(load|store|atomic)")


def mtd_instance(name):
    """(P, REF, BEAMS, JOB) of an mtd_kernel symbol, or None."""
    m = re.match(r"_ZN3rsp10mtd_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb([01])E", name)
    return tuple(int(g) for g in m.groups()) if m else None


def check_dma_wait(body, k_loads):
    """Problems with the LDS-DMA wait of one kernel body ([] = the invariant holds)."""
    dma = [i for i, s in enumerate(body) if s.startswith("buffer_load") and re.search(r"\blds\b", s)]
    if not dma:
        return None   # no LDS-DMA in this instance
    # the tile's DMA run: the pieces up to the first barrier after the first one
    bar = next((i for i in range(dma[0], len(body)) if body[i].startswith("s_barrier")), None)
    if bar is None:
        return ["no s_barrier after the LDS-DMA pieces"]
    last = max(i for i in dma if i < bar)
    probs, issued, cover = [], 0, None
    for i in range(last + 1, bar):
        s = body[i]
        if re.match(r"^s_(cbranch|branch|setpc|swappc)", s):
            probs.append("branch between the last DMA piece and the barrier: %s" % s)
        if _VMEM.match(s):
            issued += 1
        m = re.match(r"^s_waitcnt\b.*\bvmcnt\((\d+)\)", s)
        if m and cover is None and int(m.group(1)) <= issued:
            cover = (int(m.group(1)), issued)
    if cover is None:
        probs.append("the DMA pieces are not covered by any vmcnt wait before the barrier (%d VMEM issued after them)"
                     % issued)
    else:
        n, at = cover
        if n != at:
            probs.append("covering wait vmcnt(%d) with %d VMEM instructions issued after the last piece" % (n, at))
        if at != k_loads:
            probs.append("%d VMEM instructions between the last DMA piece and its wait, expected kLoads = %d"
                         % (at, k_loads))
    return probs


def run(lib=LIB, verbose=False):
    fns = functions(disassemble(lib))
    checked, bad = [], {}
    for name, body in sorted(fns.items()):
        inst = mtd_instance(name)
        if inst is None:
            continue
        P, REF, BEAMS, JOB = inst
        probs = check_dma_wait(body, K_JOB_LOADS if JOB else 0)
        if probs is None:
            continue
        checked.append(inst)
        if probs:
            bad[inst] = probs
        if verbose:
            print("mtd_kernel<%d,%d,%d,%s>: %s" % (P, REF, BEAMS, "true" if JOB else "false",
                                                   "ok" if not probs else "; ".join(probs)))
    return checked, bad


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    checked, bad = run(lib, verbose=True)
    print("%d LDS-DMA mtd_kernel instances checked, %d with problems" % (len(checked), len(bad)))
    return 1 if bad or not checked else 0


if __name__ == "__main__":
    sys.exit(main())
