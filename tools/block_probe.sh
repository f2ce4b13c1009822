set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/blk
for b in 2 4 8; do
  RRAY_BLOCK_ROWS=$b timeout -k 10 300 python tools/part_scaling.py c3_s1024_reflect 5 > gpurun_out/blk/part_b$b.json 2> gpurun_out/blk/part_b$b.err || { tail -5 gpurun_out/blk/part_b$b.err; exit 1; }
  echo "block $b"; python -c "
import json; d=json.load(open('gpurun_out/blk/part_b$b.json'))
print({k:(v['max_part_ms'],v['speedup_bound'],v['balance']) for k,v in d['parts'].items()}, d['one_part_ms'], d.get('virtual_group_8_ms'))"
done
