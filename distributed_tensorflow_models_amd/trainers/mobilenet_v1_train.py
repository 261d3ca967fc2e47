"""Entry script: reference vgg/nets/mobilenet_v1_train.py (preset ``mobilenet_v1``: SGD 0.045,
x0.94 every 2.5 epochs, batch 64, ImageNet 224, --depth_multiplier, --fine_tune_checkpoint).

``--quantize``: fake-quantised training (compat.quantize; weights and activations 8-bit after
``--quant_delay`` steps, 0 when fine-tuning - reference get_quant_delay, mobilenet_v1_train.py:66-73).
"""
from ..compat import flags
from .. import trainer

trainer.define_common_flags(flags, "mobilenet_v1")
flags.DEFINE_boolean("quantize", False, "Quantize training")
flags.DEFINE_integer("quant_delay", 250000, "steps before fake quantisation starts (training from scratch)")
flags.DEFINE_string("dataset_dir", "", "Location of dataset (alias of --data_dir)")
flags.DEFINE_integer("number_of_steps", 0, "Number of training steps (alias of --max_steps)")


def main(_argv=None):
    F = flags.FLAGS
    if F.dataset_dir:
        F.data_dir = F.dataset_dir
    if F.number_of_steps:
        F.max_steps = F.number_of_steps
    return trainer.train("mobilenet_v1", flags, default_mode="bsp")


if __name__ == "__main__":
    flags.run(main)
