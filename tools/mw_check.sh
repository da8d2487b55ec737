#!/bin/bash
# Generic kernel (bench.py --jit off) at two register budgets on scenes beyond the headline (960x540),
# and the stock config's secondary number (REFCOMPAT spp 4 depth 50 -- on the scene-specialised kernel,
# so a control: the library build changes only the generic kernel).
# usage: tools/mw_check.sh LIB_A LIB_B   (paths of librrte_hip builds; "" = the default library)
set -o pipefail
for lib in "$@"; do
  L=${lib:-rrte_amd/lib/librrte_hip.so}
  for sc in deformation-stress mesh-demo advanced-demo; do
    echo "start lib=$L scene=$sc"
    RRTE_HIP_LIB=$L timeout -k 10 240 python bench.py --jit off --no-cpu --no-stock --no-boundary --scene $sc \
      --width 960 --height 540 --steps 20 --warmup 3 > /tmp/mwc.json || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/mwc.json').read().strip().splitlines()[-1]); print('lib=$L scene=$sc generic ms/frame', d['ms_per_step'], 'u8diff', d.get('verified',{}).get('u8_max_diff'))"
  done
  echo "start lib=$L stock"
  RRTE_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu --no-boundary --steps 5 --warmup 2 > /tmp/mwc.json || exit 1
  python3 -c "import json; d=json.loads(open('/tmp/mwc.json').read().strip().splitlines()[-1]); print('lib=$L stock', d['stock_config'])"
done
