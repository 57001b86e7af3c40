"""Step watchdog detection logic (train/watchdog.py; SURVEY.md §5 failure detection) on the CPU: a step that stops
making progress fires within the timeout, steady steps never do, and idle time between steps is not counted."""
import time

from huggingface_sagemaker_tensorflow_distributed_amd.train.watchdog import StepWatchdog


def _wd(timeout, fired):
    return StepWatchdog(timeout, rank=3, describe=lambda: "phase test", poll_s=0.05,
                        on_stall=lambda r: fired.append(r)).start()


def test_stalled_step_fires_with_context():
    fired = []
    wd = _wd(0.3, fired)
    wd.step_begin(7)
    time.sleep(1.0)
    wd.stop()
    assert len(fired) == 1
    assert "rank 3" in fired[0] and "host in step 7" in fired[0] and "phase test" in fired[0]


def test_steady_steps_do_not_fire():
    fired = []
    wd = _wd(0.3, fired)
    for s in range(10):
        wd.step_begin(s)
        time.sleep(0.1)
        wd.step_end(s)
    wd.stop()
    assert fired == []


def test_idle_between_steps_is_not_counted():
    fired = []
    wd = _wd(0.3, fired)
    wd.step_begin(0)
    wd.step_end(0)
    time.sleep(0.8)  # e.g. evaluation or a checkpoint between steps
    wd.step_begin(1)
    time.sleep(0.1)
    wd.step_end(1)
    time.sleep(0.2)
    wd.stop()
    assert fired == []
