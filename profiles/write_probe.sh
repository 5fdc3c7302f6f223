#!/bin/bash
# WRITE_SIZE (KiB per dispatch, PMC) of the C2 tile kernel for several library builds.
#   bash profiles/write_probe.sh lib1.so lib2.so ...
set -u
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  out=gpurun_out/wp_$n
  VR_LIBRARY=$lib timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d "$out" -o run -- python3 profiles/profile_kernel.py --config C2 --kernel tile --iters 3 > /dev/null 2>&1 || { echo "failed: $lib"; exit 1; }
  python3 - "$out" "$n" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/*counter_collection.csv") for r in csv.DictReader(open(f))
     if "march_kernel" in r["Kernel_Name"] and "true>" not in r["Kernel_Name"]]
print(sys.argv[2], "WRITE_SIZE KiB per dispatch:", [round(x) for x in v])
PY
done
