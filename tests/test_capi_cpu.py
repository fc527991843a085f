"""CPU-side checks of the C-ABI boundary: the library loads, exports every function
include/rsp.h declares, and reports errors (no compute without a GPU)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    text = open(os.path.join(ROOT, "include", "rsp.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rsp_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header():
    from rsp import _capi
    lib = _capi.load_library()
    declared = _header_functions()
    assert len(declared) >= 10
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_capi.EXPORTS) == declared
    assert lib.rsp_version().startswith(b"rsp-mi355x")


def test_struct_layouts_match_header():
    """ctypes mirrors of rsp.h structs: sizes computed from the C compiler."""
    import subprocess
    import tempfile
    from rsp import _capi
    src = ('#include "rsp.h"\n#include <stdio.h>\nint main(void){printf("%zu %zu %zu\\n", sizeof(rsp_pc_segment),'
           ' sizeof(rsp_params), sizeof(rsp_cfar_params));return 0;}\n')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "s")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        sizes = [int(x) for x in subprocess.check_output([exe]).split()]
    assert sizes == [C.sizeof(_capi.rsp_pc_segment), C.sizeof(_capi.rsp_params), C.sizeof(_capi.rsp_cfar_params)]


def test_errors_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    from rsp import RspError, presets
    from rsp.engine import Engine
    with pytest.raises(RspError) as ei:
        Engine(presets.v2(64, 1024))
    assert ei.value.code in (5, 3)   # RSP_ERR_HIP (no device)
    from rsp import _capi
    lib = _capi.load_library()
    assert lib.rsp_last_error(None)  # the message is kept for rsp_last_error(NULL)


def test_null_arguments():
    from rsp import _capi
    lib = _capi.load_library()
    assert lib.rsp_create(None, 0, None) == _capi.RSP_ERR_ARG
    assert b"null" in lib.rsp_last_error(None)
    assert lib.rsp_destroy(None) == 0
    assert lib.rsp_pc_mtd_cfar_dev(None, None, 0, 0, None, None, None, None, None) == _capi.RSP_ERR_ARG
