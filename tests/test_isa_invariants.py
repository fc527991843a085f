"""Build-time invariant of the shipped kernels (CPU only): the MTD tile's hand-counted LDS-DMA
wait (`s_waitcnt vmcnt(Hook::kLoads)` in rsp_kernels.hip mtd_tile) covers exactly the DMA
pieces -- kLoads range-job gathers issue between the last piece and the wait, none above the
DMA -- in every mtd_kernel instance of lib/librsp.so (tools/isa_check.py)."""
import os
import re
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check  # noqa: E402

pytestmark = pytest.mark.skipif(
    not os.path.exists(isa_check.LIB) or not os.path.exists(os.path.join(isa_check.LLVM, "llvm-objdump")),
    reason="needs the built library and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def fns():
    return isa_check.functions(isa_check.disassemble())


def _body(fns, P, job):
    name = next(n for n in fns if isa_check.mtd_instance(n) == (P, 5, 1, job))
    return list(fns[name])


def test_shipped_mtd_dma_waits_hold():
    checked, bad = isa_check.run()
    assert not bad, bad
    # the bench configurations' tiles (c3 P=128, c4 P=256, c5 P=512) use the DMA path with a job
    for P in (128, 256, 512):
        assert (P, 5, 1, 1) in checked and (P, 5, 1, 0) in checked


@pytest.mark.parametrize("P", [128, 256, 512])
def test_checker_rejects_edited_counts(fns, P):
    body = _body(fns, P, 1)
    assert isa_check.check_dma_wait(body, 17) == []
    i = next(k for k, s in enumerate(body) if re.match(r"^s_waitcnt vmcnt\(17\)$", s))
    for n in (16, 18, 0):   # a count edited down over-waits (drains the gathers), up leaves the DMA uncovered
        edited = body[:i] + ["s_waitcnt vmcnt(%d)" % n] + body[i + 1:]
        assert isa_check.check_dma_wait(edited, 17), n


def test_checker_rejects_hoisted_or_merged_gather(fns):
    body = _body(fns, 128, 1)
    dma = [k for k, s in enumerate(body) if s.startswith("buffer_load") and " lds" in s]
    last = dma[len([d for d in dma if d < next(k for k, s in enumerate(body) if s.startswith("s_barrier"))]) - 1]
    g = next(k for k in range(last + 1, len(body)) if body[k].startswith("buffer_load_dword "))
    hoisted = body[:dma[0]] + [body[g]] + body[dma[0]:g] + body[g + 1:]   # one gather above the DMA
    assert isa_check.check_dma_wait(hoisted, 17)
    merged = body[:g] + body[g + 1:]                                      # one gather fewer
    assert isa_check.check_dma_wait(merged, 17)


def test_tools_present():
    assert shutil.which(os.path.join(isa_check.LLVM, "clang-offload-bundler"))
