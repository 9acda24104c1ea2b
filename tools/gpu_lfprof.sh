# cProfile of one long-form bench step (host-side time, GPU waits included)
timeout -k 10 600 python3 -m cProfile -o gpurun_out/lf.prof bench.py --mode longform --steps 1 --warmup 1 --audio-seconds 60 > gpurun_out/lf2.json 2> gpurun_out/lf2.err
echo "rc=$?"
python3 -c "import pstats; pstats.Stats('gpurun_out/lf.prof').sort_stats('tottime').print_stats(30)" > gpurun_out/lf_prof.txt
tail -45 gpurun_out/lf_prof.txt
