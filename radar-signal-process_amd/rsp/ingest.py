"""Raw-data ingest: the radar's PRT record stream -> DBF beams on the GPU.

Mirrors the reference's reader stack with the same names and argument meaning:
  * DataFullPathGen(path, fileInd)                      DataFullPathGen.m:2-27
  * FileStream.read(n) -> (data, actual, is_end)         read_continuous_file_stream.m:22-168,
    the persistent state as members and its EOF-exact branch (:138-150) kept as written: a
    read that ends exactly at a file's end advances the file index, and the next open (:48)
    advances it again, so that file's successor is skipped (quirk=False reads straight on)
  * FrameDataRead_xzr(stream, DBF_coeffs_data_C, Sig_Config, frameRInd)
        -> (sig_data_DBF_allprts, servo_angle, frameCompleted, is_global_stream_end)
    FrameDataRead_xzr.m:20-204, with the parse, the payload decode of every data type (DDC
    + DBF product, ADC, the 24-bit DBF branch) on the GPU (rsp_ingest_frame_dev,
    csrc/rsp_ingest.hip).  sig_data_DBF_allprts is a torch complex64 tensor on the device in
    the chain's layout [beam][prt][sample] (MATLAB's is prt x sample x beam: .permute(1, 2, 0)).
  * read_dbf_coeffs(path)                                bin_to_mat_xzr.m:22-29

The host reads each record as the reference does (head, realtime block, payload sized by the
head, tail, each one read through the stream and stopping where the reference returns, so the
stream position and file-boundary behaviour match) into one buffer per frame; the GPU then
locates and checks every record itself.  No CPU fallback: the parse, the decode and the
beamforming run only in librsp.so.
"""
import ctypes as C
import os

import numpy as np

from . import _capi as capi


def DataFullPathGen(DataFilePath, fileInd):  # noqa: N802 (reference name)
    """DataFullPathGen.m:10-27."""
    if fileInd < 10:
        name = "1.00000" + str(fileInd) + ".bin"
    elif fileInd < 100:
        name = "1.0000" + str(fileInd) + ".bin"
    else:
        name = "1.000" + str(fileInd) + ".bin"
    sub = os.path.join(DataFilePath, "雷达原始数据")
    return os.path.join(sub if os.path.isdir(sub) else DataFilePath, name)


class FileStream:
    """read_continuous_file_stream.m: a byte stream over 1.00000k.bin files, k = 1, 2, ..."""

    def __init__(self, orgDataFilePath, quirk=True):
        self.path = orgDataFilePath
        self.quirk = quirk
        self._f = None
        self._pos = 0
        self._size = 0
        self._index = 0

    def _open_next(self):
        self._index += 1
        try:
            f = open(DataFullPathGen(self.path, self._index), "rb")
        except OSError:
            self._f = None
            return False
        self._size = os.fstat(f.fileno()).st_size
        self._f, self._pos = f, 0
        return True

    def _close(self):
        if self._f is not None:
            self._f.close()
        self._f = None

    def read(self, n):
        """(bytes, actual length, is_end_of_stream)."""
        if self._f is None and not self._open_next():
            return b"", 0, True
        if self._pos + n > self._size:                 # straddles into the next file
            data = self._f.read(max(self._size - self._pos, 0))
            self._close()
            if n - len(data) > 0:
                if not self._open_next():
                    self._pos = self._size = 0
                    return data, len(data), True
                more = self._f.read(n - len(data))
                self._pos += len(more)
                data += more
        elif self._pos + n == self._size:              # ends exactly at EOF
            data = self._f.read(n)
            self._close()
            if self.quirk:
                self._index += 1
            self._pos = self._size = 0
        else:
            data = self._f.read(n)
            self._pos += len(data)
        return data, len(data), len(data) < n and self._f is not None

    def close(self):
        self._close()


class BytesStream:
    """An in-memory record stream with FileStream's read contract."""

    def __init__(self, data):
        self._data = memoryview(bytes(data))
        self._pos = 0

    def read(self, n):
        part = bytes(self._data[self._pos:self._pos + n])
        self._pos += len(part)
        return part, len(part), len(part) < n


def read_dbf_coeffs(path):
    """bin_to_mat_xzr.m:22-29: comma/space separated rows, columns alternating I, Q per
    channel -> beam x channel complex128."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.replace(",", " ").strip()
            if line:
                rows.append([float(v) for v in line.split()])
    m = np.asarray(rows, dtype=np.float64)
    return m[:, 0::2] + 1j * m[:, 1::2]


def payload_bytes(data_type, pdn, ch):
    """FrameDataRead_xzr.m:105-119: a record's signal bytes by data type, padded to 64 B."""
    if data_type == 0:
        sig = pdn * ch * 2
    elif data_type == 1:
        sig = pdn * ch * 4
    else:
        sig = pdn * ch * 6 + pdn * (8 - (6 * ch) % 8)
    return sig + (64 - sig % 64 if sig % 64 else 0)


def dbf24_values(ch):
    """Values per sample row of the 24-bit DBF branch (:132-133, three column ranges), or -1
    where MATLAB raises a size error (unequal ranges or an odd count at :163)."""
    L = 6 * ch + (8 - (6 * ch) % 8)
    n1, n2, n3 = len(range(0, L - 3, 3)), len(range(1, L - 2, 3)), len(range(2, L, 3))
    return n1 if n1 == n2 == n3 and n1 % 2 == 0 else -1


def _shape_ok(data_type, pdn, ch, cfg):
    """Whether the reference gets past :171-176 (and :158's inner dimension for DDC) -- the host
    needs it only to stop reading where the reference does (before the tail).  Types 3..255
    match no case of :160-165, so their row stays zeros(point_PRT, beam_num) and always passes."""
    if data_type > 2:
        return True
    if pdn != cfg["point_PRT"]:
        return False
    if data_type == 1:
        return ch == cfg["channel_num"]
    if data_type == 0:
        return ch == cfg["beam_num"]
    return dbf24_values(ch) == 2 * cfg["beam_num"]


def sig_config(prtNum=332, point_PRT=3404, channel_num=16, beam_num=13, bytesFrameHead=64,  # noqa: N803
               bytesFrameEnd=64, bytesFrameRealtime=128, fs=100e6, timer_freq=200e6):
    """bin_to_mat_xzr.m:35-43 (field names as there)."""
    return dict(fs=fs, timer_freq=timer_freq, prtNum=prtNum, point_PRT=point_PRT, channel_num=channel_num,
                beam_num=beam_num, bytesFrameHead=bytesFrameHead, bytesFrameEnd=bytesFrameEnd,
                bytesFrameRealtime=bytesFrameRealtime)


class Ingest:
    """GPU frame decoder: owns an rsp context (CFAR-only kind: no chain parameters needed)
    and the device buffers of one frame."""

    def __init__(self, device=0):
        import torch
        self.lib = capi.load_library()
        self.device = torch.device("cuda", device)
        ctx = C.c_void_p()
        capi.check(self.lib.rsp_create(C.byref(ctx), int(device), None), None)
        self.ctx = ctx
        self._state = {}          # the device copy of the last DBF coefficient matrix

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.rsp_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def params(cfg):
        p = capi.rsp_ingest_params()
        p.prt_num, p.point_prt = cfg["prtNum"], cfg["point_PRT"]
        p.channel_num, p.beam_num = cfg["channel_num"], cfg["beam_num"]
        p.bytes_head, p.bytes_realtime, p.bytes_tail = cfg["bytesFrameHead"], cfg["bytesFrameRealtime"], cfg["bytesFrameEnd"]
        return p

    def record_bytes(self, cfg):
        n = C.c_int64()
        capi.check(self.lib.rsp_ingest_record_bytes(C.byref(self.params(cfg)), C.byref(n)), None)
        return n.value

    def dbf_device(self, dbf_C):
        """beam x channel complex -> device float32 [beam][channel][2]."""
        import torch
        d = np.ascontiguousarray(np.stack([np.real(dbf_C), np.imag(dbf_C)], axis=-1), dtype=np.float32)
        return torch.from_numpy(d).to(self.device)

    def decode_dev(self, d_stream, nbytes, cfg, d_dbf, out=None, beam_stride=0, stream=None, ddc_only=False):
        """rsp_ingest_frame_dev (every data type, records sized by their heads) or, ddc_only,
        rsp_ingest_ddc_dev on device buffers; returns (out, servo uint16, status int32)."""
        import torch
        P, R, B = cfg["prtNum"], cfg["point_PRT"], cfg["beam_num"]
        if out is None:
            out = torch.empty((B, P, R), dtype=torch.complex64, device=self.device)
        servo = torch.empty((P,), dtype=torch.int16, device=self.device)
        status = torch.empty((P + 1,), dtype=torch.int32, device=self.device)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        fn = self.lib.rsp_ingest_ddc_dev if ddc_only else self.lib.rsp_ingest_frame_dev
        capi.check(fn(
            self.ctx, C.c_void_p(d_stream.data_ptr()), int(nbytes), C.byref(self.params(cfg)),
            C.c_void_p(d_dbf.data_ptr()), C.c_void_p(out.data_ptr()), int(beam_stride),
            C.c_void_p(servo.data_ptr()), C.c_void_p(status.data_ptr()), C.c_void_p(s.cuda_stream)), self.ctx)
        return out, servo, status

    @staticmethod
    def read_frame_bytes(stream, cfg):
        """The frame's records as the reference reads them (FrameDataRead_xzr.m:57-189: head,
        then -- unless pulse_data_num is 0 -- realtime block, payload sized by the head's type,
        samples and channels, and -- unless the size check fails -- tail), stopping where it
        returns.  Returns (bytes, stream_ended)."""
        bh, br, bt = cfg["bytesFrameHead"], cfg["bytesFrameRealtime"], cfg["bytesFrameEnd"]
        parts = []

        def take(n):
            data, got, end = stream.read(n)
            parts.append(data)
            return not (end or got < n)

        for _ in range(cfg["prtNum"]):
            if not take(bh):
                return b"".join(parts), True
            head = np.frombuffer(parts[-1][:32], dtype="<u4")
            pdn, ch, typ = int(head[6]), int(head[3] & 0xff), int(head[7] & 0xff)
            if pdn == 0 or not take(br) or not take(payload_bytes(typ, pdn, ch)):
                return b"".join(parts), True
            if not _shape_ok(typ, pdn, ch, cfg) or not take(bt):
                return b"".join(parts), True
        return b"".join(parts), False

    def FrameDataRead_xzr(self, stream, DBF_coeffs_data_C, Sig_Config, frameRInd):  # noqa: N802,N803
        """FrameDataRead_xzr.m:20-204 -> (beams [beam][prt][sample] complex64 on the GPU,
        servo_angle float64 [prt] (host), frameCompleted, is_global_stream_end)."""
        import torch
        data, _ = self.read_frame_bytes(stream, Sig_Config)
        d_stream = torch.frombuffer(bytearray(data) if data else bytearray(1), dtype=torch.uint8).to(self.device)
        key = np.ascontiguousarray(DBF_coeffs_data_C, dtype=np.complex128).tobytes()
        if self._state.get("dbf_key") != key:
            self._state["dbf"] = self.dbf_device(np.asarray(DBF_coeffs_data_C))
            self._state["dbf_key"] = key
        out, servo, status = self.decode_dev(d_stream, len(data), Sig_Config, self._state["dbf"])
        st = status.cpu().numpy()
        P = Sig_Config["prtNum"]
        stop = int(st[P])
        completed = stop == P and not np.any(st[:P] == capi.RSP_PRT_TAIL_TRUNCATED)
        angles = servo.cpu().numpy().view(np.uint16).astype(np.float64)
        # every early return of the reference sets is_global_stream_end (:62-189); a
        # completed frame returns (true, false) (:201-202)
        return out, angles, bool(completed), bool(not completed)
