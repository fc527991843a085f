"""GPU tests of the sliding-window stream and of the fused
range-CFAR variants of the chain (flagV not requested; rFlag = 0).

Window i of frame pair (n, n+1) is rows [round(i*P/win), +P) of [frame n; frame n+1]
(MTD/main_produce_dataset_win_xzr_v2.m:117-131).  Pulse compression is row-wise, so the
engine computes each frame's PC once and every window reads it: the windowed outputs must be
BIT-identical to the plain chain run on the sliced echo, and within the RDM / CFAR bars of
SURVEY.md §8d against the fp64 oracle.
"""
import numpy as np
import pytest

from _util import NEAR_TOL, RDM_TOL, flag_mismatch, oracle_flags, oracle_rdm, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def _mround(x):
    return int(np.floor(x + 0.5))


def _windows(frames, win):
    """[beams, F+1, P, R] -> [beams, F, win, P, R] by the reference's slicing."""
    beams, nf1, P, R = frames.shape
    out = np.empty((beams, nf1 - 1, win, P, R), dtype=frames.dtype)
    for b in range(beams):
        for n in range(nf1 - 1):
            pair = np.concatenate([frames[b, n], frames[b, n + 1]], axis=0)
            for i in range(win):
                s = _mround(i * P / win)
                out[b, n, i] = pair[s:s + P]
    return out


@pytest.mark.parametrize("P,R,beams,nf,win,chunk,streams,prefilter", [
    (64, 1024, 2, 3, 4, 0, 0, False), (128, 4096, 1, 2, 4, 0, 0, False), (64, 1024, 1, 5, 3, 8, 0, False),
    (96, 1024, 1, 2, 5, 0, 0, False),
    # several chunks on two pipelines (two scratch slots, each chunk with its look-ahead frame)
    (64, 1024, 1, 7, 4, 8, 2, False), (64, 1024, 2, 5, 3, 3, 2, False),
    # the fused pre-filters (iSTC gain in PC's load, MTI lag 9 in the MTD's load) in window mode
    (64, 1024, 1, 4, 4, 0, 0, True), (64, 1024, 1, 5, 4, 8, 2, True)])
def test_window_bit_exact_vs_sliced_chain(torch_cuda, P, R, beams, nf, win, chunk, streams, prefilter):
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    eng = Engine(spec, device=0, chunk=chunk, streams=streams)
    if prefilter:
        eng.set_prefilter(gain=np.linspace(0.5, 2.0, R).astype(np.float32), mti_lag=9)
    cf = presets.default_cfar(spec)
    frames = synth.echo_numpy(spec, beams * (nf + 1), seed=1004).reshape(beams, nf + 1, P, R)
    d_frames = torch.from_numpy(frames).cuda()
    shp = (beams, nf, win, P, spec.R_out)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.window_dev(d_frames, win, rdm=d_rdm, flag=d_flag, cfar=cf)
    sliced = _windows(frames, win).reshape(-1, P, R)
    d_sl = torch.from_numpy(np.ascontiguousarray(sliced)).cuda()
    n = sliced.shape[0]
    e_rdm = torch.empty((n, P, spec.R_out), dtype=torch.float32, device="cuda")
    e_flag = torch.empty((n, P, spec.R_out), dtype=torch.uint8, device="cuda")
    eng.run_dev(d_sl, rdm=e_rdm, flag=e_flag, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(d_rdm.reshape(n, P, -1), e_rdm)
    assert torch.equal(d_flag.reshape(n, P, -1), e_flag)
    eng.close()


def test_window_parity_vs_oracle(torch_cuda):
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R, win = 64, 1024, 4
    spec = presets.v2(P, R)
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    frames = synth.echo_numpy(spec, 3, seed=1044).reshape(1, 3, P, R)
    d_frames = torch.from_numpy(frames).cuda()
    shp = (1, 2, win, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.window_dev(d_frames, win, rdm=d_rdm, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    sliced = _windows(frames, win).reshape(-1, P, R)
    rdm = oracle_rdm("v2", sliced)
    got = d_rdm.cpu().numpy().reshape(-1, P, R)
    assert rel_err(got, rdm) < RDM_TOL
    flag, _, amb = oracle_flags(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy().reshape(-1, P, R), flag, amb)
    assert hard == 0 and soft <= 2, (hard, soft)
    assert flag.sum() > 0
    # window 0 of pair n is frame n itself
    assert rel_err(got[0], oracle_rdm("v2", frames[0, :1])[0]) < RDM_TOL
    eng.close()


def test_window_errors(torch_cuda):
    torch = torch_cuda
    from rsp import presets
    from rsp._capi import RspError
    from rsp.engine import Engine
    eng = Engine(presets.v2(64, 1024), device=0)
    d = torch.zeros((1, 2, 64, 1024), dtype=torch.complex64, device="cuda")
    r = torch.empty((1, 1, 17, 64, 1024), dtype=torch.float32, device="cuda")
    with pytest.raises(RspError):
        eng.window_dev(d, 17, rdm=r)         # win > 16
    with pytest.raises(ValueError):
        eng.window_dev(d[:, :1].contiguous(), 4, rdm=r)   # needs >= 2 frames
    eng.close()


def test_chain_without_flagV_matches(torch_cuda):
    """The hot path (flagV not requested: no Doppler-flag plane is written) gives the same
    flags as the path that also returns flagV."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    for P, R in ((64, 1024), (128, 4096)):
        spec = presets.v2(P, R)
        eng = Engine(spec, device=0)
        cf = presets.default_cfar(spec)
        echo = torch.from_numpy(synth.echo_numpy(spec, 3, seed=1005)).cuda()
        shp = (3, P, R)
        f1 = torch.empty(shp, dtype=torch.uint8, device="cuda")
        f2 = torch.empty(shp, dtype=torch.uint8, device="cuda")
        fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
        r1 = torch.empty(shp, dtype=torch.float32, device="cuda")
        eng.run_dev(echo, rdm=r1, flag=f1, cfar=cf)
        eng.run_dev(echo, flag=f2, flagV=fv, cfar=cf)     # internal RDM buffer
        torch.cuda.synchronize()
        assert torch.equal(f1, f2)
        assert int(f1.sum()) > 0 and int(fv.sum()) > int(f1.sum())
        eng.close()


def test_chain_rflag0_is_flagV(torch_cuda):
    """rCFARDetect_Flag = 0: executeCFAR returns flag = flagV (executeCFAR.m:91)."""
    torch = torch_cuda
    import dataclasses
    from rsp import presets, synth
    from rsp.engine import Engine
    P, R = 64, 1024
    spec = presets.v2(P, R)
    eng = Engine(spec, device=0)
    cf = dataclasses.replace(presets.default_cfar(spec), rFlag=0)
    echo_np = synth.echo_numpy(spec, 2, seed=1006)
    echo = torch.from_numpy(echo_np).cuda()
    shp = (2, P, R)
    f = torch.empty(shp, dtype=torch.uint8, device="cuda")
    fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
    rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    eng.run_dev(echo, rdm=rdm, flag=f, flagV=fv, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(f, fv)
    ordm = oracle_rdm("v2", echo_np)
    flag, flagV, amb = oracle_flags(ordm, cf)
    assert np.array_equal(flag, flagV)
    hard, soft = flag_mismatch(f.cpu().numpy(), flag, amb)
    assert hard == 0 and soft <= 2
    eng.close()


def test_dmx_native_two_beam_parity(torch_cuda):
    """Row a8: the DMX chain at native size (1536 PRTs x 566 samples, two beams): PC (raw FIR
    short part + circular 512-point MF), fft(pc.*hamming, 2048, 1), |L|+|R| with the
    zeroSetFlagMTD rows, |R|-|L|, executeCFAR per short/long part on the sum.  Bars: sum
    rel-err <= 1e-5; diff error <= 1e-5 of the sum's norm (it is a difference of magnitudes);
    flags exact outside the near-threshold band."""
    torch = torch_cuda
    import rsp_ref as ref
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.dmx_native()
    assert spec.R_out == 574 and spec.V == 2048 and spec.radar["M0"] == 6
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    batch = 2
    rng = np.random.default_rng(1008)
    e = (rng.standard_normal((batch, 2, spec.P, spec.R)) + 1j * rng.standard_normal((batch, 2, spec.P, spec.R))) \
        * np.sqrt(0.5)
    # moving targets in both beams (different gains): the replica itself, delayed into the
    # long part, with a per-PRT Doppler phase -- it compresses to a range/Doppler peak
    rep = presets.load_data("refDDCDataMF1").astype(np.complex128).ravel()
    m = np.arange(spec.P)[:, None]
    for delay, fd, amp in ((150, 0.11, 0.5), (320, -0.23, 0.3)):
        sig = amp * np.exp(2j * np.pi * fd * m) * rep[None, :] / np.abs(rep).max()
        c0 = 62 + delay
        e[:, 0, :, c0:c0 + rep.size] += sig
        e[:, 1, :, c0:c0 + rep.size] += 0.6 * sig
    e = e.astype(np.complex64)
    d_in = torch.from_numpy(e).cuda()
    shp = (batch, spec.V, spec.R_out)
    d_sum = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_diff = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_sum, diff=d_diff, flag=d_flag, cfar=cf)
    torch.cuda.synchronize()
    H = ref.dmx_matched_filter(presets.load_data("refDDCDataMF1"), 512)
    sums, diffs = [], []
    for b in range(batch):
        pcl = ref.dmx_pulse_compression(e[b, 0].astype(np.complex128), 62, 512, H)
        pcr = ref.dmx_pulse_compression(e[b, 1].astype(np.complex128), 62, 512, H)
        s, d = ref.dmx_mtd_pair(pcl, pcr, 2048, spec.radar["M0"])
        sums.append(s)
        diffs.append(d)
    s_ref, d_ref = np.stack(sums), np.stack(diffs)
    assert rel_err(d_sum.cpu().numpy(), s_ref) < RDM_TOL
    assert np.linalg.norm(d_diff.cpu().numpy() - d_ref) / np.linalg.norm(s_ref) < RDM_TOL
    flag, _, amb = oracle_flags(s_ref, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    assert hard == 0 and soft <= 2, (hard, soft)
    assert flag.sum() > 0
    eng.close()


@pytest.mark.parametrize("P,R,batch", [(332, 3404, 2), (100, 1024, 2), (75, 1024, 1)])
def test_bluestein_mtd_parity(torch_cuda, P, R, batch):
    """Pulse counts without a radix plan -- the v2 native 332 x 3404 CPI
    (MTD/main_produce_dataset_win_xzr_v2.m:31,37) and an odd P -- run the slow-time DFT by
    Bluestein's identity.  RDM rel-err <= 1e-5 against the fp64 oracle's direct DFT; CFAR
    exact outside the near-threshold band."""
    torch = torch_cuda
    from rsp import presets, synth
    from rsp.engine import Engine
    spec = presets.v2(P, R)
    eng = Engine(spec, device=0)
    cf = presets.default_cfar(spec)
    echo = synth.echo_numpy(spec, batch, seed=1009)
    d_in = torch.from_numpy(echo).cuda()
    shp = (batch, P, R)
    d_rdm = torch.empty(shp, dtype=torch.float32, device="cuda")
    d_flag = torch.empty(shp, dtype=torch.uint8, device="cuda")
    d_fv = torch.empty(shp, dtype=torch.uint8, device="cuda")
    eng.run_dev(d_in, rdm=d_rdm, flag=d_flag, flagV=d_fv, cfar=cf)
    torch.cuda.synchronize()
    rdm = oracle_rdm("v2", echo)
    assert rel_err(d_rdm.cpu().numpy(), rdm) < RDM_TOL
    flag, flagV, amb = oracle_flags(rdm, cf)
    hard, soft = flag_mismatch(d_flag.cpu().numpy(), flag, amb)
    hardv, softv = flag_mismatch(d_fv.cpu().numpy(), flagV, amb)
    assert hard == 0 and hardv == 0, (hard, hardv)
    assert soft <= 2 and softv <= 2
    assert flagV.sum() > 0
    eng.close()


def test_window_stream_with_range_concat(torch_cuda):
    """The sliding-window stream (rsp_window_pc_mtd_cfar_dev) on a context with main.m's range
    concatenation (rsp_set_range_concat): each frame's PC is computed once at the full 1031
    columns, gathered to 868, and every window reads its rows from the gathered frame -- bit-exact
    against the chain on the explicitly sliced windows of the same context."""
    torch = torch_cuda
    from rsp import presets
    from rsp.engine import Engine
    spec = presets.legacy(64, 1031, concat=True)
    cf = presets.default_cfar(spec)
    eng = Engine(spec)
    F, win, P = 3, 4, 64
    from rsp import synth
    frames = synth.echo_torch(spec, F + 1, seed=77).reshape(1, F + 1, P, 1031)
    rdm = torch.empty((1, F, win, P, 868), dtype=torch.float32, device="cuda")
    flag = torch.empty((1, F, win, P, 868), dtype=torch.uint8, device="cuda")
    eng.window_dev(frames, win, rdm=rdm, flag=flag, cfar=cf)
    torch.cuda.synchronize()
    for n in range(F):
        pair = torch.cat([frames[0, n], frames[0, n + 1]], dim=0)
        wins = torch.stack([pair[_mround(i * P / win):_mround(i * P / win) + P] for i in range(win)]).contiguous()
        r2 = torch.empty((win, P, 868), dtype=torch.float32, device="cuda")
        f2 = torch.empty((win, P, 868), dtype=torch.uint8, device="cuda")
        eng.run_dev(wins, rdm=r2, flag=f2, cfar=cf)
        torch.cuda.synchronize()
        assert torch.equal(r2, rdm[0, n]) and torch.equal(f2, flag[0, n]), n
    # one frame pair per chunk on two pipelines: each pipeline gathers from its own full-width slot
    eng.set_chunk(win)
    eng.set_streams(2)
    r3 = torch.empty_like(rdm)
    f3 = torch.empty_like(flag)
    eng.window_dev(frames, win, rdm=r3, flag=f3, cfar=cf)
    torch.cuda.synchronize()
    assert torch.equal(r3, rdm) and torch.equal(f3, flag)
    eng.close()
