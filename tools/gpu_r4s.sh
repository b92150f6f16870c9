# Round-4 session s: per-phase refinement profile, session start vs now.
mkdir -p gpurun_out
for v in r4start qflag tmpl; do
  ALVRL_LIB=mitsuba-alvrl_amd/variants/libalvrl_$v.so ALVRL_REFINE_PROFILE=1 ALVRL_REFINE_TEAM_STATS=1 timeout -k 10 200 python -u bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --no-alt > gpurun_out/r4s_$v.json 2> gpurun_out/r4s_$v.err || exit 1
done
