OLD="OFLOW_LIB=$PWD/build/rev_head/_lib/liboflow_hip.so OFLOW_OPS_LIB=$PWD/build/rev_head/_lib/liboflow_torch.so"
tools/gpu_job.sh \
 "400|r3_s2_pytest|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_corr_convc1.py tests/test_gpu_raft.py tests/test_gpu_conv_s32.py" \
 "120|r3_s2_stamps|python -u tools/exp/run_convc1_stamps.py" \
 "200|r3_s2_ab|for i in 1 2; do env $OLD python -u tools/exp/step_ab.py; python -u tools/exp/step_ab.py; done"
