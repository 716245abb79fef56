set -o pipefail
mkdir -p gpurun_out
for sd in 32 16 8 64; do
  timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-recall --opt sample_div=$sd > gpurun_out/sd_$sd.json 2>gpurun_out/sd_$sd.err || { tail gpurun_out/sd_$sd.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sd_$sd.json'));r=d['roofline'];print('c2 sd $sd',d['value'],d['ms_per_step'],r['avg_launch_ms'],d['search_stats'])"
done
for sd in 32 16; do
  timeout -k 10 300 python -u bench.py --config nstar --steps 10 --no-cpu-baseline --no-recall --opt sample_div=$sd > gpurun_out/sdn_$sd.json 2>gpurun_out/sdn_$sd.err || { tail gpurun_out/sdn_$sd.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sdn_$sd.json'));r=d['roofline'];print('nstar sd $sd',d['value'],d['ms_per_step'],r['avg_launch_ms'],d['search_stats'])"
done
