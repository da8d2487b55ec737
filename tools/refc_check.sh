#!/bin/bash
# REFCOMPAT on the generic kernel (bench.py --jit off) for two library builds: the default (REFCOMPAT
# variants at 5 waves) and one given (e.g. every variant at 6 waves); single-sample and the stock config.
set -o pipefail
for lib in "" "$1"; do
  L=${lib:-rrte_amd/lib/librrte_hip.so}
  for cfgargs in "--mode refcompat" "--mode refcompat --spp 4 --max-depth 50 --random"; do
    echo "start lib=$L $cfgargs"
    RRTE_HIP_LIB=$L timeout -k 10 240 python bench.py --jit off --no-cpu --no-stock --no-boundary $cfgargs \
      --width 960 --height 540 --steps 20 --warmup 3 > /tmp/rc.json || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/rc.json').read().strip().splitlines()[-1]); print('lib=$L [$cfgargs] generic ms/frame', d['ms_per_step'], 'u8diff', d.get('verified',{}).get('u8_max_diff'))"
  done
done
