"""The reference's matplotlib figures (ref src/train.py:43-57,111-117; src/train_dist.py:49-56).

Only rank 0 writes (the reference lets every rank overwrite the same PNG,
SURVEY.md section 5.2).  matplotlib is optional: without it the plot calls are
no-ops that return False.
"""
from __future__ import annotations

from pathlib import Path


def _plt():
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        return plt
    except Exception:
        return None


def plot_loss_curve(train_counter, train_losses, test_counter, test_losses, path) -> bool:
    plt = _plt()
    if plt is None:
        return False
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    fig = plt.figure()
    plt.plot(train_counter, train_losses, color="blue")
    plt.scatter(test_counter[: len(test_losses)], test_losses, color="red")
    plt.legend(["Train Loss", "Test Loss"], loc="upper right")
    plt.xlabel("number of training examples seen")
    plt.ylabel("negative log likelihood loss")
    fig.savefig(path)
    plt.close(fig)
    return True


def plot_examples(images, labels, path, n: int = 6) -> bool:
    """2x3 grid of sample digits with their labels (ref src/train.py:43-57)."""
    plt = _plt()
    if plt is None:
        return False
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    fig = plt.figure()
    for i in range(min(n, len(images))):
        plt.subplot(2, 3, i + 1)
        plt.tight_layout()
        plt.imshow(images[i].reshape(28, 28), cmap="gray", interpolation="none")
        plt.title("Ground Truth: {}".format(int(labels[i])))
        plt.xticks([])
        plt.yticks([])
    fig.savefig(path)
    plt.close(fig)
    return True


def plot_scaling(gpus, times, path, title="Time to train (1 epoch) vs. Number of GPUs") -> bool:
    plt = _plt()
    if plt is None:
        return False
    Path(path).parent.mkdir(parents=True, exist_ok=True)
    fig = plt.figure()
    plt.plot(gpus, times, marker="o")
    plt.xlabel("number of GPUs")
    plt.ylabel("seconds")
    plt.title(title)
    fig.savefig(path)
    plt.close(fig)
    return True
