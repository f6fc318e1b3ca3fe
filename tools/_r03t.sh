# Last check of the final tree: GPU tests, smoke, the default bench command (the driver's).
steps=(pytest 900 "python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 5 --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'"
       bench_default 400 "python bench.py")
bash tools/gpu_steps.sh r03t "${steps[@]}"
