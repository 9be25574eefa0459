cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for w in 5 5 50; do
  timeout -k 10 300 python bench.py --steps 20 --warmup $w --no-cpu --host-calls 0 --no-sweep > gpurun_out/b_w$w.log 2>&1 || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/b_w$w.log'):
    if l.startswith('{'):
        d=json.loads(l); o=d['ops']
        print('warmup $w', d['value'], d['ms_per_step'], 'enc', o['encode_ms'], 'A timed', o['decode_stageA_ms'], 'A bd', o['decode_stageA_breakdown_ms'], 'B', o['decode_stageB_ms'], 'setup', o['decode_setup_ms'])
"
done
