#!/bin/bash
# (superseded by tools/runs/r03_kinds.sh, which reports the per-launch times too)
true
