mkdir -p gpurun_out/r06e
timeout -k 10 300 python -u tools/search_image_breakdown.py > gpurun_out/r06e/search_image.json 2> gpurun_out/r06e/err.log && timeout -k 10 300 python -u tools/search_image_breakdown.py --profile > gpurun_out/r06e/profile.txt 2>> gpurun_out/r06e/err.log; rc=$?; cat gpurun_out/r06e/search_image.json; exit $rc
