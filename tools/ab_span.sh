export TMPDIR=/tmp EBPF_BUCKET=1
mkdir -p gpurun_out/r03e
for w in 1 2 4; do
  for e in "" ; do
    EBPF_SPAN_WAVES=$w timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03e/kt$w -o kt -- python3 bench.py --config c5 --also= --no-cpu-baseline --no-pmc --no-verify --steps 20 --warmup 5 > gpurun_out/r03e/b$w.json 2>gpurun_out/r03e/b$w.err || exit 1
    echo "== waves $w"; python3 tools/kt_summary.py gpurun_out/r03e/kt$w 5 | tail -6
  done
done
