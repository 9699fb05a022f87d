"""Host-side guard of the whole-step HIP graph (graphs.hw_queue_problem): with fewer than 4 hardware
queues per process (GPU_MAX_HW_QUEUES) the HIP runtime segfaulted inside hipGraphLaunch replaying the
multi-stream step graph (profiles/r6/hw_queues_ab.log), so bench.py --graph and train.py --hip-graph
refuse it and --compile falls back to eager with the reason logged."""
from fault_tolerant_llm_training_amd.graphs import hw_queue_problem


def test_hw_queue_guard(monkeypatch):
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert hw_queue_problem() == ""
    for q in ("4", "8", "32"):
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", q)
        assert hw_queue_problem() == ""
    for q in ("1", "2", "3"):
        monkeypatch.setenv("GPU_MAX_HW_QUEUES", q)
        assert "GPU_MAX_HW_QUEUES=" + q in hw_queue_problem()
