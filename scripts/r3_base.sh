set -e
mkdir -p gpurun_out/r3base
for spec in "q3:--config q3" "q6:--config q6" "q6f32:--config q6f32" "q6pert:--config q6 --perturb 0.1" "q3dofmap:--config q3 --kernel dofmap --geometry stored"; do
  name=${spec%%:*}; args=${spec#*:}
  echo "== $name"
  timeout -k 10 240 python bench.py $args --steps 50 --warmup 5 --extras off > gpurun_out/r3base/$name.json 2> gpurun_out/r3base/$name.err
  python -c "import json;d=json.load(open('gpurun_out/r3base/$name.json'));print('$name',d['value'],d['ms_per_step'],d['config']['kernel'])"
done
