import sys, os, time, torch
sys.path[:0] = ["radar-signal-process_amd", "tests/golden"]
from make_golden_ingest import synth_frame
from rsp import ingest
_, dbf, _, cfg, rec = synth_frame(332, 3404, 16, 13, seed=1)
ing = ingest.Ingest(0)
d = torch.frombuffer(bytearray(rec), dtype=torch.uint8).cuda()
dd = ing.dbf_device(dbf)
out = torch.empty((13, 332, 3404), dtype=torch.complex64, device="cuda")
for mode in (False, True, False, True):
    for _ in range(5): ing.decode_dev(d, len(rec), cfg, dd, out=out, ddc_only=mode)
    torch.cuda.synchronize(); e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(50): ing.decode_dev(d, len(rec), cfg, dd, out=out, ddc_only=mode)
    e1.record(); torch.cuda.synchronize()
    print("ddc_only" if mode else "frame   ", round(e0.elapsed_time(e1) / 50 * 1e3, 2), "us/frame")
