#!/bin/bash
# HBM bytes of the multifrontal solve's leaf launches (mf_fwd_kernel / mf_bwd_kernel over the 17k leaf
# fronts, 1M convection-diffusion): one FETCH_SIZE pass and one kernel-trace pass of tools/mf_probe.py,
# joined per dispatch for the largest-grid mf_fwd / mf_bwd launches
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/r6/leafpmc $R/gpurun_out/r6/leaftr
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r6/leafpmc -o pmc -- python3 $R/tools/mf_probe.py 1000 > $R/gpurun_out/r6/leafpmc.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r6/leaftr -o tr -- python3 $R/tools/mf_probe.py 1000 > $R/gpurun_out/r6/leaftr.log 2>&1 || exit 1
cd $R
python3 - <<'PY'
import csv, glob, collections
pm = glob.glob('gpurun_out/r6/leafpmc/**/*counter_collection.csv', recursive=True)[0]
tr = glob.glob('gpurun_out/r6/leaftr/**/*kernel_trace.csv', recursive=True)[0]
fetch = collections.defaultdict(list)
for r in csv.DictReader(open(pm)):
    k = r['Kernel_Name'].split('(')[0]
    g = int(r.get('Grid_Size', r.get('Grid_Size_X', 0)) or 0)
    fetch[(k, g)].append(float(r['Counter_Value']))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(tr)):
    k = r['Kernel_Name'].split('(')[0]
    g = int(r['Grid_Size_X']) * int(r.get('Grid_Size_Y', 1) or 1)
    dur[(k, g)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for key in sorted(set(fetch) & set(dur), key=lambda x: -max(dur[x])):
    if 'mf_' not in key[0]:
        continue
    f = sum(fetch[key]) / len(fetch[key]); d = sum(dur[key]) / len(dur[key])
    print(f"{key[0][-40:]:40s} grid {key[1]:9d}  {len(dur[key]):4d} x {d:8.1f} us  FETCH_SIZE {f/1e3:10.1f} MB(raw kB units?)  rate {f*1e3/ (d*1e-6) / 1e12 if d else 0:.2f}")
PY
