"""Log-line formats and loss series of the reference trainers.

* single-process train line (ref src/train.py:78-80)
* single-process test line  (ref src/train.py:100-104)
* distributed epoch summary (ref src/train_dist.py:113-114, including the
  literal spaces produced by the backslash continuation inside the f-string)
"""
from __future__ import annotations

from dataclasses import dataclass, field


def train_line(epoch: int, seen: int, total: int, pct: float, loss: float) -> str:
    return "Train Epoch: {} [{}/{} ({:.0f}%)]\tLoss: {:.6f}".format(epoch, seen, total, pct, loss)


def test_line(avg_loss: float, correct: int, total: int, elapsed: float) -> str:
    return "\nTest set: Avg. loss: {:.4f}, Accuracy: {}/{} ({:.0f}%), time_elapsed={:.4f}\n".format(
        avg_loss, correct, total, 100.0 * correct / total, elapsed)


def dist_epoch_line(epoch: int, train_loss: float, val_loss: float, accuracy: float, elapsed: float) -> str:
    return (f"Epoch={epoch}, train_loss={train_loss:.4f}, val_loss={val_loss:.4f}, accuracy={accuracy:.2f}, "
            f"          time_elapsed={elapsed:.4f}")


@dataclass
class LossHistory:
    """train_losses / train_counter / test_losses / test_counter of the reference."""
    train_losses: list = field(default_factory=list)
    train_counter: list = field(default_factory=list)
    test_losses: list = field(default_factory=list)
    test_counter: list = field(default_factory=list)
