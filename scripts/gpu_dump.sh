cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dump
for i in 1 2 3 4; do
  LM_DUMP_DIR=gpurun_out/dump timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batch 512 --resident 6400 > gpurun_out/dump/b$i.json 2> gpurun_out/dump/b$i.err
  rc=$?; echo "run $i rc=$rc $(grep -o 'checkVel.*' gpurun_out/dump/b$i.err | head -1)"
  [ $rc -ne 0 ] && break
done
ls gpurun_out/dump
