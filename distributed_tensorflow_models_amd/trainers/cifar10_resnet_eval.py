"""Evaluator: reference resnet/cifar10_resnet_eval.py (preset ``resnet``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "resnet")


def main(_argv=None):
    evaluator.evaluate("resnet", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
