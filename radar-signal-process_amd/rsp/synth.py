"""Deterministic synthetic echoes, the input of tests and the benchmark.

    x[m, n] = sum_t A_t * s_seg(t)[n - d_t] * exp(j*2*pi*f_dt*m*PRT) + c[n] + w[m, n]

  w ~ CN(0, 1) (I and Q each N(0, 1/2)); A_t = 10^(SNR/20) with SNR = 20 dB; one target
  per pulse-compression segment with velocities -5.7 m/s (MatlabProcess_xuzerui/main.m:186),
  +12 m/s and -20 m/s (f_d = 2v/lambda); target 1 at the 320 m delay of main.m:187;
  zero-Doppler clutter c[n], +30 dB over noise with a random phase, on the first R/8 bins
  (exercises fun_0v_pressing).  The waveform of a segment is the replica its matched filter
  uses (a 4-sample pulse for the FIR segment).  numpy's PCG64 with seed = base + CPI index
  makes every CPI reproducible on any host; `echo_torch` draws the noise on the GPU instead
  (same recipe, a different random stream) for benchmark-sized batches.
"""
import math

import numpy as np

from . import _capi as capi

VELOCITIES = (-5.7, 12.0, -20.0)


def _targets(spec):
    """[(waveform, delay_column, velocity)] for a spec."""
    rp = spec.radar
    deltaR = rp.get("deltaR", 2.99792458e8 / (2 * rp.get("fs", 25e6)))
    out = []
    segs = spec.segments
    if len(segs) == 1:
        s = segs[0]
        wf = np.asarray(s.coef, np.complex128)
        wf = wf / np.max(np.abs(wf))
        for i, v in enumerate(VELOCITIES):
            d = s.in_start + int(round(s.in_len * (0.2 + 0.3 * i)))
            out.append((wf, d, v))
        return out
    for i, s in enumerate(segs[:3]):
        v = VELOCITIES[i % 3]
        if s.kind == capi.RSP_SEG_FIR:
            wf = np.ones(4, np.complex128)
            d = int(round(320.0 / deltaR))
            if d + 4 > s.in_len:
                d = s.in_len // 3
        else:
            wf = np.asarray(s.coef, np.complex128)
            wf = wf / np.max(np.abs(wf))
            d = s.in_len // 7 if i == 1 else s.in_len // 2
        out.append((wf, s.in_start + d, v))
    return out


def _clean(spec, snr_db=20.0):
    """Target part of one CPI (deterministic, no noise): P x R complex128."""
    P, R = spec.P, spec.R
    rp = spec.radar
    lam, prt = rp["wavelength"], rp["prt"]
    x = np.zeros((P, R), np.complex128)
    amp = 10.0 ** (snr_db / 20.0)
    m = np.arange(P)
    for wf, d, v in _targets(spec):
        fd = 2.0 * v / lam
        dop = np.exp(1j * 2.0 * np.pi * fd * m * prt)
        n = min(len(wf), R - d)
        if n > 0:
            x[:, d:d + n] += amp * np.outer(dop, wf[:n])
    return x


def _clutter(spec, rng):
    R = spec.R
    nc = max(1, R // 8)
    phase = rng.uniform(0, 2 * np.pi, nc)
    c = np.zeros(R, np.complex128)
    c[:nc] = 10.0 ** (30.0 / 20.0) * np.exp(1j * phase)
    return c


def echo_numpy(spec, batch=1, seed=1000, dtype=np.complex64, snr_db=20.0, scale=1.0):
    """[batch, P, R] synthetic echoes; CPI b uses numpy PCG64(seed + b).  snr_db: target
    power over the unit noise power; scale multiplies the whole echo (fp16 range sweeps)."""
    P, R = spec.P, spec.R
    clean = _clean(spec, snr_db)
    out = np.empty((batch, P, R), dtype)
    for b in range(batch):
        rng = np.random.Generator(np.random.PCG64(seed + b))
        w = (rng.standard_normal((P, R)) + 1j * rng.standard_normal((P, R))) * math.sqrt(0.5)
        x = clean + _clutter(spec, rng)[None, :] + w
        out[b] = x * scale if scale != 1.0 else x
    return out


def to_half_iq(echo):
    """complex array [..., P, R] -> float16 [..., P, R, 2] (unit noise power: no overflow; the
    tolerance sweep's largest scales go past the fp16 range on purpose and become +-inf, as a
    float16 store does)."""
    e = np.asarray(echo)
    out = np.empty(e.shape + (2,), np.float16)
    with np.errstate(over="ignore"):
        out[..., 0] = e.real
        out[..., 1] = e.imag
    return out


def echo_torch(spec, batch, seed=1000, device="cuda", half=False):
    """Benchmark-sized batch generated on the GPU: [batch, P, R] complex64, or
    [batch, P, R, 2] float16 when half=True."""
    import torch
    P, R = spec.P, spec.R
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    base = torch.from_numpy(_clean(spec).astype(np.complex64)).to(device)
    rng = np.random.Generator(np.random.PCG64(seed))
    clut = torch.from_numpy(_clutter(spec, rng).astype(np.complex64)).to(device)
    fixed = base + clut[None, :]
    if half:
        out = torch.empty((batch, P, R, 2), dtype=torch.float16, device=device)
    else:
        out = torch.empty((batch, P, R), dtype=torch.complex64, device=device)
    step = max(1, (256 << 20) // (P * R * 8))
    for b0 in range(0, batch, step):
        n = min(step, batch - b0)
        w = torch.randn((n, P, R, 2), generator=g, device=device, dtype=torch.float32) * math.sqrt(0.5)
        x = torch.view_as_complex(w) + fixed[None]
        if half:
            out[b0:b0 + n] = torch.view_as_real(x).to(torch.float16)
        else:
            out[b0:b0 + n] = x
    return out
