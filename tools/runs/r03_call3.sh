#!/bin/bash
set -o pipefail
bash tools/r03_ab.sh "" "-DRRTE_MARCH_PRED=1" || exit 1
bash tools/runs/r03_verify.sh
