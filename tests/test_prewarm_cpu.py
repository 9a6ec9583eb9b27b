"""train.py's restart VRAM warm-up: only on a relaunch (DLGM_RESTART > 0) with the previous attempt's engine size
recorded under the save dir; the thread ends on its own (no GPU here: hipSetDevice fails and it returns)."""
from distributed_llm_training_gpu_manager_amd import train


def test_prewarm_only_on_relaunch_with_a_recorded_size(tmp_path, monkeypatch):
    argv = ["--model", "llama-tiny", "--save-dir", str(tmp_path)]
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("DLGM_RESTART", "0")
    assert train.start_prewarm(argv) is None  # first launch
    monkeypatch.setenv("DLGM_RESTART", "1")
    assert train.start_prewarm(argv) is None  # nothing recorded yet
    (tmp_path / ".engine_vram_gib.r0").write_text("1.5")
    th = train.start_prewarm(argv)
    assert th is not None
    th.join(timeout=60)
    assert not th.is_alive()
    assert train.start_prewarm(["--save-dir=" + str(tmp_path)]) is not None
    monkeypatch.setenv("RANK", "3")
    assert train.start_prewarm(argv) is None  # another rank's record is not this rank's
