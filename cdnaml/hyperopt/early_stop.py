"""Early-stop callbacks for ``fmin(early_stop_fn=...)``."""
from __future__ import annotations


def no_progress_loss(iteration_stop_count: int = 20, percent_increase: float = 0.0):
    def stop_fn(trials, best_loss=None, iteration_no_progress=0):
        new_loss = trials.trials[-1]["result"].get("loss") if len(trials) else None
        if best_loss is None:
            return False, [new_loss, iteration_no_progress + 1]
        if new_loss is not None and new_loss < best_loss - abs(best_loss) * percent_increase / 100.0:
            best_loss, iteration_no_progress = new_loss, 0
        else:
            iteration_no_progress += 1
        return iteration_no_progress >= iteration_stop_count, [best_loss, iteration_no_progress]
    return stop_fn
