"""Evaluator: reference cnn/cifar10_eval.py (preset ``cnn``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "cnn")


def main(_argv=None):
    evaluator.evaluate("cnn", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
