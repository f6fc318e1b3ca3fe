steps=(pytest 900 "python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 5 --timeout 300 --timeout-method thread"
       smoke 200 "python -c 'import __graft_entry__ as g; g.smoke()'")
bash tools/gpu_steps.sh r03j "${steps[@]}" && bash tools/_r03i.sh
