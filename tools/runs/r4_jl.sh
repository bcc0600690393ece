#!/bin/bash
set -o pipefail
bash tools/runs/r4_j.sh && bash tools/runs/r4_l.sh
