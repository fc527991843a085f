"""The reference's MATLAB entry points, same names, same argument meaning, same outputs.

    MTD_Signal = fun_MTD_produce(echoData, params)            MTD/fun_MTD_produce.m:12
    MTD_Signal = fun_MTD_produce_legacy(echo)                  MatlabProcess_xuzerui/fun_MTD_produce.m:3
    [flag, flagV] = executeCFAR(rdm, refR, saveR, TR, mR,
                                refV, saveV, TV, mV, M0, rFlag)   CFAR_WangCai/executeCFAR.m:1-2
    cfarFlag = fun_CFARflag(rdm, ... same 10 scalars ...)      CFAR_WangCai/main_cfar.m:142

Arrays follow MATLAB conventions: echoData is P x R complex (rows = PRTs), outputs are
float64 (RDM magnitude, flags 0/1).  A numpy C-order P x R array is passed row-major;
the engine also accepts MATLAB column-major buffers (see Engine.pc_mtd_cfar).
Error behaviour: where MATLAB raises (an index error for a CFAR window that does not fit,
a size mismatch), these raise rsp._capi.RspError.
All computation runs on the GPU through librsp; nothing here computes on the CPU.
"""
import numpy as np

from . import _capi as capi
from . import presets
from .engine import Engine

_engines = {}


def _engine(key, make_spec, device=0):
    e = _engines.get(key)
    if e is None:
        e = Engine(make_spec(), device=device)
        _engines[key] = e
    return e


def _params_key(params, P, R):
    pp = tuple(params["point_prt"])
    return ("v2", P, R, pp, params["fs"], params["B"], tuple(params["tao"]))


def fun_MTD_produce(echoData, params, device=0):
    """MTD/fun_MTD_produce.m:12-158: PC (fun_lss_pulse_compression) -> MTD
    (fun_Process_MTD) -> fun_0v_pressing.  echoData: P x R complex."""
    echo = np.asarray(echoData)
    if echo.ndim != 2:
        raise ValueError("echoData must be P x R")
    P, R = echo.shape
    rp = dict(params)
    rp.setdefault("prtNum", P)
    if int(rp["point_prt"][0]) != R:
        # MATLAB uses the array's own width for segment 3 (fun_lss_pulse_compression.m:20-25)
        rp["point_prt"] = [R] + list(rp["point_prt"][1:])
    eng = _engine(_params_key(rp, P, R), lambda: presets.v2(P, R, radar=_full_radar(rp, P, R)), device)
    return eng.pc_mtd(echo.astype(np.complex128, copy=False)[None])[0].astype(np.float64)


def _full_radar(rp, P, R):
    full = presets.radar_params(P, R, rp["point_prt"], fs=rp["fs"], fc=rp.get("fc", 9450e6),
                                prt=rp.get("prt", 232.76e-6), B=rp["B"], tao=rp["tao"])
    return full


def fun_MTD_produce_legacy(echo, device=0):
    """MatlabProcess_xuzerui/fun_MTD_produce.m:3-126 (1-argument legacy form)."""
    e = np.asarray(echo)
    P, R = e.shape
    eng = _engine(("legacy", P, R), lambda: presets.legacy(P, R), device)
    return eng.pc_mtd(e.astype(np.complex128, copy=False)[None])[0].astype(np.float64)


def _cfar_engine(device=0):
    # rsp_cfar needs a context only for its device and buffers: rsp_create(params=NULL)
    return _engine(("cfar-only",), lambda: None, device)


def executeCFAR(echo_MTD, refCells_R, saveCells_R, T_CFAR_R, CFARmethod_R, refCells_V, saveCells_V,
                T_CFAR_V, CFARmethod_V, MTD_0_num, rCFARDetect_Flag, device=0):
    """CFAR_WangCai/executeCFAR.m:1-93 -> (cfarResultFlag_Matrix, cfarResultFlag_MatrixV)."""
    rdm = np.asarray(echo_MTD, dtype=np.float64)
    cf = presets.Cfar(refR=int(refCells_R), saveR=int(saveCells_R), TR=float(T_CFAR_R),
                      methodR=int(CFARmethod_R), refV=int(refCells_V), saveV=int(saveCells_V),
                      TV=float(T_CFAR_V), methodV=int(CFARmethod_V), M0=int(MTD_0_num),
                      rFlag=int(bool(rCFARDetect_Flag)), zero_v_div=0, segments=[])
    flag, flagV = _cfar_engine(device).cfar(rdm.astype(np.float32)[None], cf)
    return flag[0].astype(np.float64), flagV[0].astype(np.float64)


def fun_CFARflag(MTD_data, refCells_R, saveCells_R, T_CFAR_R, CFARmethod_R, refCells_V, saveCells_V,
                 T_CFAR_V, CFARmethod_V, MTD_0_num, rCFARDetect_Flag,
                 segments=((0, 82), (82, 318), (318, 868)), device=0):
    """CFAR_WangCai/main_cfar.m:142-161: executeCFAR per column segment (default the
    hard-coded 1:82 | 83:318 | 319:868), columns outside every segment stay 0."""
    rdm = np.asarray(MTD_data, dtype=np.float64)
    cf = presets.Cfar(refR=int(refCells_R), saveR=int(saveCells_R), TR=float(T_CFAR_R),
                      methodR=int(CFARmethod_R), refV=int(refCells_V), saveV=int(saveCells_V),
                      TV=float(T_CFAR_V), methodV=int(CFARmethod_V), M0=int(MTD_0_num),
                      rFlag=int(bool(rCFARDetect_Flag)), zero_v_div=0, segments=list(segments))
    flag, _ = _cfar_engine(device).cfar(rdm.astype(np.float32)[None], cf)
    return flag[0].astype(np.float64)
