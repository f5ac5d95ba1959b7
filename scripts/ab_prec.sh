mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest default rc=$?"; tail -1 gpurun_out/pytest_gpu.log
FAISS_AMD_IVF_PREC=bf16x3 timeout -k 10 600 python -m pytest tests/test_gpu_flat_ivf.py tests/test_gpu_golden.py -q -m gpu -x > gpurun_out/pytest_bf3.log 2>&1; echo "pytest bf16x3 rc=$?"; tail -1 gpurun_out/pytest_bf3.log
FAISS_AMD_IVF_STATS=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --recall-queries 0 2>&1 | grep "ivf mfma"
FAISS_AMD_IVF_PREC=bf16x3 timeout -k 10 300 python bench.py --no-cpu-baseline --recall-queries 0 > gpurun_out/b3.json 2>/dev/null; echo "bf16x3: $(python -c "import json;d=json.load(open('gpurun_out/b3.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])")"
timeout -k 10 300 python bench.py --no-cpu-baseline --recall-queries 0 > gpurun_out/b2.json 2>/dev/null; echo "bf16x2: $(python -c "import json;d=json.load(open('gpurun_out/b2.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])")"
