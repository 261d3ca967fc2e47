"""Evaluator: reference vgg/nets/mobilenet_v1_eval.py (preset ``mobilenet_v1``; top-1 / top-5 over
the ImageNet validation split, --depth_multiplier)."""
from ..compat import flags
from .. import evaluator

evaluator.define_eval_flags(flags, "mobilenet_v1")
flags.DEFINE_float("depth_multiplier", 1.0, "Depth multiplier for mobilenet")
flags.DEFINE_string("dataset_dir", "", "Location of dataset (alias of --data_dir)")
flags.DEFINE_boolean("quantize", False, "Quantize training (evaluate the fake-quantised graph)")


def main(_argv=None):
    F = flags.FLAGS
    if F.dataset_dir:
        F.data_dir = F.dataset_dir
    evaluator.evaluate("mobilenet_v1", flags)
    return 0


if __name__ == "__main__":
    flags.run(main)
