# summary of a gpu_fc16.sh run: tests tail, bench lines, update stamps
T=$1
cd /root/repo/gpurun_out
tail -3 ${T}_tests.log
for f in ${T}_bench_lb ${T}_bench_1024 ${T}_bench_64 ${T}_bench_8; do
  [ -f $f.log ] && python -c "
import json
l=[x for x in open('$f.log') if x.startswith('{')][-1]; d=json.loads(l); print('$f', round(d['ms_per_step']*1000,2), d['value'], d['config'].get('device_ms_per_step'))"
done
grep -v amdgpu ${T}_upd.log 2>/dev/null
