"""Evaluator: reference cifarnet/cifar10_cifarnet_eval.py (preset ``cifarnet``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "cifarnet")


def main(_argv=None):
    evaluator.evaluate("cifarnet", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
