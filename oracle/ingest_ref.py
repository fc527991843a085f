"""oracle/ingest_ref.py -- TEST INFRASTRUCTURE ONLY.

fp64 numpy restatement of the reference's raw-data ingest, the checker of
the HIP ingest path (radar-signal-process_amd/csrc/rsp_ingest.hip):
  * DataFullPathGen.m:2-27            file naming  '1.00000<k>.bin' / '1.0000<k>' / '1.000<k>'
  * read_continuous_file_stream.m:22-168   the cross-file byte stream, including its
    EOF-exact branch (:138-150) that advances the file index once more than needed, so the
    next open (:47-48) skips a file -- restated as written;
  * FrameDataRead_xzr.m:20-204        per-PRT record parse (head fields :70-86, sizes
    :104-119), int16 I/Q DDC decode (:149-156) and DBF sig_data_C * DBF_coeffs_data_C.'
    (:158), the ADC matrix (:144-147), the 24-bit DBF branch (:130-135,162-164) with MATLAB's
    uint8 arithmetic (saturating products and sums, as the reference evaluates it), frame
    bookkeeping (persistent current_prt / last_frameRInd, :23-52), the early returns and the
    size check (:171-176).
Also the inverse: `prt_record` writes a record in that format, which the tests use to build
.bin streams (the reference ships neither .bin captures nor its DBF coefficient file,
bin_to_mat_xzr.m:23).  Parity is therefore "parity unpinned" beyond this restatement: no
reference fixture holds ingest outputs.  Nothing in the product imports this module.
"""
import os

import numpy as np

HEAD_WORDS = 16


def data_full_path_gen(path, file_ind):
    """DataFullPathGen.m:10-27 (the optional '雷达原始数据' subdirectory included)."""
    if file_ind < 10:
        name = "1.00000%d.bin" % file_ind
    elif file_ind < 100:
        name = "1.0000%d.bin" % file_ind
    else:
        name = "1.000%d.bin" % file_ind
    sub = os.path.join(path, "雷达原始数据")
    return os.path.join(sub if os.path.isdir(sub) else path, name)


class ContinuousFileStream:
    """read_continuous_file_stream.m as an object (its persistent variables, :25-40)."""

    def __init__(self, root):
        self.root = root
        self.is_open = False
        self.f = None
        self.pos = 0
        self.max_len = 0
        self.index = 0

    def _open(self, ind):
        name = data_full_path_gen(self.root, ind)
        try:
            f = open(name, "rb")
        except OSError:
            return False
        f.seek(0, 2)
        self.max_len = f.tell()
        f.seek(0)
        self.f, self.pos, self.is_open = f, 0, True
        return True

    def read(self, n):
        """(data bytes, actual length, is_end_of_stream) -- :22-168."""
        data = b""
        if not self.is_open:                                    # :47-69
            self.index += 1
            if not self._open(self.index):
                return data, 0, True
        if self.pos + n > self.max_len:                         # :81-135 straddles a boundary
            part = self.f.read(max(self.max_len - self.pos, 0))
            data = part
            self.f.close()
            self.f, self.is_open = None, False
            remain = n - len(data)
            if remain > 0:
                self.index += 1
                if not self._open(self.index):
                    self.pos, self.max_len = 0, 0
                    return data, len(data), True
                part = self.f.read(remain)
                data += part
                self.pos += len(part)
        elif self.pos + n == self.max_len:                      # :138-150 ends exactly at EOF
            data = self.f.read(n)
            self.f.close()
            self.f, self.is_open = None, False
            self.index += 1                                      # (and :48 adds one more on the next open)
            self.pos, self.max_len = 0, 0
        else:                                                    # :153-158
            data = self.f.read(n)
            self.pos += len(data)
        if len(data) < n and self.is_open:                      # :163-166
            return data, len(data), True
        return data, len(data), False


def dbf_from_text(rows):
    """bin_to_mat_xzr.m:27-29: columns alternate I, Q per channel -> beam x channel complex."""
    m = np.asarray(rows, dtype=np.float64)
    return m[:, 0::2] + 1j * m[:, 1::2]


def ddc_payload_bytes(point, channels):
    """FrameDataRead_xzr.m:108-119 for data_type 1: samples * channels * 2 * 2, padded to 64 B."""
    return payload_bytes(1, point, channels)


def payload_bytes(data_type, pdn, ch):
    """FrameDataRead_xzr.m:105-119: signal bytes by data type, padded to 64 B."""
    if data_type == 0:
        sig = pdn * ch * 2
    elif data_type == 1:
        sig = pdn * ch * 2 * 2
    else:
        sig = pdn * ch * 2 * 3 + pdn * (8 - (6 * ch) % 8)
    return sig + (64 - sig % 64 if sig % 64 else 0)


def _u8(x):
    """MATLAB uint8 result of a double-valued expression: round, then saturate."""
    return np.clip(np.round(x), 0, 255)


def dbf24_parse(raw, pdn, ch):
    """FrameDataRead_xzr.m:130-135 as MATLAB runs it (data_temp is uint8, so every product and
    sum saturates) and :163 (value pairs -> I/Q columns).  Raises ValueError where MATLAB raises
    a size error (column ranges of unequal length, or an odd value count)."""
    pad = 8 - (6 * ch) % 8                                                    # :111
    L = ch * 2 * 3 + pad
    t = np.frombuffer(raw[:pdn * L], dtype=np.uint8).reshape(pdn, L).astype(np.float64)   # :132
    c1, c2, c3 = t[:, 0:L - 3:3], t[:, 1:L - 2:3], t[:, 2:L:3]               # 1:3:end-3, 2:3:end-2, 3:3:end
    if not (c1.shape == c2.shape == c3.shape):
        raise ValueError("matrix dimensions must agree (:133)")
    parsed = _u8(_u8(c1 + _u8(c2 * 2 ** 8)) + _u8(c3 * 2 ** 16))             # :133
    neg = parsed > 2 ** 23                                                   # :134-135 (never, in uint8)
    parsed[neg] = _u8(parsed[neg] - 2 ** 24)
    if parsed.shape[1] % 2:
        raise ValueError("matrix dimensions must agree (:163)")
    return parsed[:, 0::2] + 1j * parsed[:, 1::2]                            # :163


def prt_record(iq, frame_no=0, pulse_no=0, servo=0, data_type=1, pulse_num=332, radar_type=2,
               timer=0, dots=(4, 200, 700), cfg=None, pulse_data_num=None, channels=None, payload=None):
    """One PRT record (the format FrameDataRead_xzr.m:61-189 parses).  iq: int16
    [samples][channels][2] (I, Q) for DDC; payload: the signal bytes of another data type
    (ADC int16 [samples][channels], DBF 24-bit rows), with iq giving only (samples, channels)."""
    cfg = cfg or {}
    bh, br, bt = cfg.get("bytesFrameHead", 64), cfg.get("bytesFrameRealtime", 128), cfg.get("bytesFrameEnd", 64)
    iq = np.asarray(iq, dtype=np.int16) if payload is None else np.asarray(iq)
    n, ch = iq.shape[0], iq.shape[1]
    head = np.zeros(bh // 4, dtype=np.uint32)
    head[0] = frame_no
    head[2] = pulse_no & 0xffff
    head[3] = (channels if channels is not None else ch) & 0xff
    head[4] = servo & 0xffff
    head[6] = n if pulse_data_num is None else pulse_data_num
    head[7] = (data_type & 0xff) | ((pulse_num & 0xffff) << 8) | ((radar_type & 0xff) << 24)
    head[8] = timer & 0xffffffff
    head[9] = (timer >> 32) & 0xffffffff
    head[10] = (dots[0] & 0xffff) | ((dots[1] & 0xffff) << 16)
    head[11] = dots[2] & 0xffff
    if payload is None:
        payload = iq.astype("<i2").tobytes()
    pad = payload_bytes(data_type, n, ch) - len(payload)
    return (head.astype("<u4").tobytes() + bytes(br) + payload + bytes(pad) +
            np.full(bt, 0xAB, dtype=np.uint8).tobytes())


class FrameReader:
    """FrameDataRead_xzr.m:20-204 with its persistent state (:23-25) as members."""

    def __init__(self):
        self.current_prt = None
        self.last_frame = None

    def read(self, stream, dbf_C, cfg, frame_ind):
        prt_num, point, beams = cfg["prtNum"], cfg["point_PRT"], cfg["beam_num"]
        bh, br, bt = cfg["bytesFrameHead"], cfg["bytesFrameRealtime"], cfg["bytesFrameEnd"]
        out = np.zeros((prt_num, point, beams), dtype=np.complex128)          # :43
        servo = np.zeros(prt_num, dtype=np.float64)                           # :44
        if self.current_prt is None or self.last_frame is None or self.last_frame != frame_ind:   # :49-52
            self.current_prt = 0
            self.last_frame = frame_ind
        while self.current_prt < prt_num:                                      # :57
            raw, n, end = stream.read(bh)                                      # :62
            if end or n < bh:
                return out, servo, False, True
            head = np.frombuffer(raw, dtype="<u4")
            ch = int(head[3] % 2 ** 8)                                         # :77
            angle = int(head[4] % 2 ** 16)                                     # :78
            pdn = int(head[6])                                                 # :79
            dtype = int(head[7] % 2 ** 8)                                      # :80
            if pdn <= 0:                                                       # :90-94
                return out, servo, False, True
            raw, n, end = stream.read(br)                                      # :97
            if end or n < br:
                return out, servo, False, True
            size = payload_bytes(dtype, pdn, ch)                               # :105-119
            raw, n, end = stream.read(size)                                    # :122
            if end or n < size:
                return out, servo, False, True
            if dtype == 0:                                                     # :144-147
                cur = np.frombuffer(raw[:pdn * ch * 2], dtype="<i2").reshape(pdn, ch).astype(np.float64)
            elif dtype == 2:                                                   # :130-135,162-164
                cur = dbf24_parse(raw, pdn, ch)
            elif dtype > 2:                                                    # :141 typecast only; no
                cur = np.zeros((point, beams), dtype=np.complex128)            # switch case (:160-165)
            else:
                words = np.frombuffer(raw[:pdn * ch * 4], dtype="<i2").astype(np.float64)   # :138,150
                sd = words.reshape(pdn, ch * 2)                                # :151
                sig_C = sd[:, 0::2] + 1j * sd[:, 1::2]                        # :154-156
                if sig_C.shape[1] != dbf_C.shape[1]:
                    raise ValueError("inner matrix dimensions must agree (:158)")
                cur = sig_C @ dbf_C.T                                          # :158
            if cur.shape != (point, beams):                                    # :171-176
                return out, servo, False, True
            self.current_prt += 1                                              # :179-181
            out[self.current_prt - 1] = cur
            servo[self.current_prt - 1] = angle
            raw, n, end = stream.read(bt)                                      # :184-189
            if end or n < bt:
                return out, servo, False, True
        return out, servo, True, False                                         # :201-202


class BytesStream:
    """A byte string as a read_continuous_file_stream-shaped source (one file, no quirk)."""

    def __init__(self, data):
        self.data = data
        self.pos = 0

    def read(self, n):
        part = self.data[self.pos:self.pos + n]
        self.pos += len(part)
        return part, len(part), len(part) < n
