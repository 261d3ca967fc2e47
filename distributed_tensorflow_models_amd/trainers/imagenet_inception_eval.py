"""Evaluator: reference inception/inception_eval.py (preset ``inception``)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "inception")


def main(_argv=None):
    evaluator.evaluate("inception", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
