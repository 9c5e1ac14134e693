#!/bin/bash
# Summary of a scripts/archive/gpu_abk1.sh run.
tail -1 gpurun_out/ab_pytest_v1.log
for f in gpurun_out/ab_*_[12].log; do echo -n "$f "; grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,2), round(d['roofline']['kernel_ms']*1000,1), 'us')"; done
paste <(grep -v '^{' gpurun_out/ab_op_base.log | awk '{print $1, $6}') <(grep -v '^{' gpurun_out/ab_op_v1.log | awk '{print $6}')
