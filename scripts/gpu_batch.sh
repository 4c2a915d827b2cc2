cd $GRAFT_REPO_ROOT
summ='import json,sys; d=json.load(sys.stdin); r=d["roofline"]; print(d["config"]["batch_frames"], d["value"], "corr_ms", r["avg_launch_ms"], "per_frame_us", round(r["avg_launch_ms"]*1000/d["config"]["batch_frames"],3), "TF", r["achieved"])'
for b in 128 256 512 1024; do
  echo -n "batch $b: "; timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --batch $b --resident 6400 2>gpurun_out/batch_$b.err | python -c "$summ" || { tail -3 gpurun_out/batch_$b.err; exit 1; }
done
