set -o pipefail
out=gpurun_out/r03d_bench
mkdir -p $out
step() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 -u bench.py "$@" > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; grep '^{' "$out/$name.log" > "$out/$name.json"; return $rc; }
step cfg3_pass 300 --steps 20 --warmup 3 &&
step cfg3_solve 300 --mode solve --steps 5 --warmup 1 --no-cpu-baseline &&
step cfg2_solve 300 --config cfg2 --mode solve --steps 20 --warmup 3 --no-cpu-baseline &&
step ladybug_pass 300 --config ladybug --steps 10 --warmup 2 &&
step cfg3_fallbacks 300 --steps 10 --warmup 2 --no-cpu-baseline --time-fallbacks
