import sys, re, statistics as st
rows = [l for l in open(sys.argv[1]) if l.startswith("rsp_host_trace")]
keys = ["setup","stage_in","enqueue","stage_out","sync","total","h2d","chain","d2h"]
vals = {k: [] for k in keys}
for l in rows:
    f = l.split()
    for k in keys:
        i = f.index(k); vals[k].append(float(f[i+1]))
print(len(rows), {k: round(st.median(v),1) for k, v in vals.items() if v})
