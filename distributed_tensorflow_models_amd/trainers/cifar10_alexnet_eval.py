"""Evaluator: reference alexnet/cifar10_alexnet_eval.py (preset ``alexnet``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "alexnet")


def main(_argv=None):
    evaluator.evaluate("alexnet", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
