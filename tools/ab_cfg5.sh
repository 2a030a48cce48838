# cfg5 replay A/B on one box: tools/build/old (an exported older tree with its own
# libvlgba.so) against the working tree, alternated twice
set -o pipefail
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then d=tools/build/old; else d=.; fi
    (cd $d && timeout -k 10 300 python -u bench.py --config cfg5 --no-cpu-baseline > /tmp/b5_$v.json 2>/tmp/b5_$v.log) || { tail -5 /tmp/b5_$v.log; exit 1; }
    python -c "
import json; d=json.load(open('/tmp/b5_$v.json')); print('$v', $r, round(d['value'],1), {k: round(v,4) for k,v in d['host_device_split_s'].items()})"
  done
done
