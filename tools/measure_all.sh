#!/bin/bash
# Round-end measurement of every bench config (tools/measure_cfg.sh: bench line, rocprofv3 stats
# on 2 and 1 pipelines, PMC; SQ counter groups for c3 and c5).
set -u
SQ=1 bash tools/measure_cfg.sh c3 && SQ=1 bash tools/measure_cfg.sh c5 && bash tools/measure_cfg.sh c2 && bash tools/measure_cfg.sh c4
