set -o pipefail
O=gpurun_out/fif; mkdir -p $O
for c in C2 C5; do for f in 2 3 4; do for s in "20 5" "200 10"; do set -- $s
timeout -k 10 120 python bench.py --config $c --frames-in-flight $f --steps $1 --warmup $2 --no-cpu-baseline > $O/${c}_f${f}_s$1.json 2>$O/err.log || exit 1
python -c "import json;d=json.load(open('$O/${c}_f${f}_s$1.json'));print('$c f=$f steps=$1', d['value'], d['ms_per_step'])"
done; done; done
