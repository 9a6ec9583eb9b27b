# side-stream wait test, then two negative controls on this box's copy (waits removed -> the test must fail)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -m gpu -q --timeout 200 --timeout-method thread -k side_stream > $O/pytest_side.log 2>&1; echo "normal rc=$?" >> $O/side_negctl.txt
tail -2 $O/pytest_side.log >> $O/side_negctl.txt
cp distributed_llm_training_gpu_manager_amd/models/mixtral.py /tmp/mix.bak
sed -i 's/                cur.wait_event(ev)/                pass  # negative control/' distributed_llm_training_gpu_manager_amd/models/mixtral.py
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -m gpu -q --timeout 200 --timeout-method thread -k "side_stream and mixtral" > $O/pytest_side_neg1.log 2>&1; echo "no-wait moe_dw rc=$?" >> $O/side_negctl.txt
cp /tmp/mix.bak distributed_llm_training_gpu_manager_amd/models/mixtral.py
sed -i 's/                torch.cuda.current_stream(self.device).wait_event(ev)$/                pass  # negative control/' distributed_llm_training_gpu_manager_amd/parallel/zero.py
grep -c "negative control" distributed_llm_training_gpu_manager_amd/parallel/zero.py >> $O/side_negctl.txt
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -m gpu -q --timeout 200 --timeout-method thread -k "side_stream and llama" > $O/pytest_side_neg2.log 2>&1; echo "no-wait tcache rc=$?" >> $O/side_negctl.txt
cat $O/side_negctl.txt
