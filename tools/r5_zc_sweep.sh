#!/bin/bash
# One-chunk (zero-copy staging) host path: MEX-granularity rate and phase trace per dev knob
# setting (rsp_capi.cpp host_chain_small): RSP_HOST_ZC 0 (DMA pipeline) / 1 (coherent staging) /
# 2 (non-coherent), RSP_ZC_PART_KIB (output part size), RSP_ZC_PIECE_KIB (input piece).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"
OUT="$ROOT/gpurun_out/zc"; mkdir -p "$OUT"
# CFGS: space-separated zc:part_kib:piece_kib triples
for cfg in ${CFGS:-1:1024:1024 0:1024:1024 2:1024:1024 1:512:1024 1:2048:1024}; do
  set -- ${cfg//:/ }
  tag="zc$1_p$2_k$3"
  RSP_HOST_ZC=$1 RSP_ZC_PART_KIB=$2 RSP_ZC_PIECE_KIB=$3 timeout -k 10 120 python tools/mex_bench.py --seconds 1.5 --trace \
      > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -3 "$OUT/$tag.err"; exit $rc; }
  echo "$tag $(python -c "import json,sys; d=json.load(open('$OUT/$tag.json')); print(d['fun_MTD_produce']['current']['calls_per_s'], d['executeCFAR']['current']['frames_per_s'])") $(python tools/parse_host_trace.py "$OUT/$tag.err")"
done
