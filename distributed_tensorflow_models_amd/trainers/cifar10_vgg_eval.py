"""Evaluator: reference (none in the reference; same contract as C56) (preset ``vgg``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "vgg")


def main(_argv=None):
    evaluator.evaluate("vgg", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
