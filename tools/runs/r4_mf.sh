#!/bin/bash
set -o pipefail
bash tools/runs/r4_m.sh && bash tools/runs/r4_final.sh
