import json, glob, sys
for f in sorted(glob.glob('gpurun_out/ablate/*.json')):
    l = [x for x in open(f) if x.startswith('{')]
    if not l:
        print(f, 'no output'); continue
    d = json.loads(l[-1]); k = d['roofline']['kernels']
    print("%-28s %9.1f  %s" % (f.split('/')[-1], d['value'], {n: v['avg_us'] for n, v in k.items()}))
