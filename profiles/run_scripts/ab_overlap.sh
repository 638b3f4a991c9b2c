set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r02o
for i in 1 2 3; do
  for m in no-overlap overlap; do
    timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu --$m > gpurun_out/r02o/$m$i.json 2> gpurun_out/r02o/$m$i.err
    python -c "import json,sys;d=json.load(open('gpurun_out/r02o/$m$i.json'));print('$m', round(d['value']/1e6,4), round(d['ms_per_step'],2), round(d['decode_kernel_ms'],2), d.get('parity_spot_check'), d['ber']['bit_errors'])"
  done
done
