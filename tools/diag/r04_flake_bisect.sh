# which preceding tests make the Mixtral EP-4 overlapped-optimizer case differ (numerical mismatch, not a fault)
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
K='swiglu or moe or mixtral or expert or mlp'
T=tests/test_shadow_async_gpu.py::test_overlapped_optimizer_waits_per_group
run() { echo "== $1"; shift; timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider "$@" 2>&1 | grep -E "passed|failed" ; }
(cd ab_old && run "old tree, same selection" tests -m gpu -x -k "$K")
run "shadow file only" tests/test_shadow_async_gpu.py -k "mixtral"
run "engine_numerics mixtral + target" tests/test_engine_numerics.py "$T" -k "mixtral"
run "kernels + target" tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py "$T" -k "swiglu or moe or mixtral"
run "mesh + target" tests/test_mesh_engine_gpu.py "$T" -k "mixtral"
run "dw_layout + target" tests/test_moe_dw_layout.py "$T" -k "gpu or mixtral"
