export TESTS="tests/test_gpu_e2e.py::test_solo_tail_bitwise tests/test_gpu_e2e.py::test_fl_rounds_on_gpu tests/test_gpu_e2e.py::test_gpu_rounds_bitwise_reproducible tests/test_gpu_e2e.py::test_fp32_eval_argmax_warm_model"
bash scripts/gpu/r4_bnx.sh
