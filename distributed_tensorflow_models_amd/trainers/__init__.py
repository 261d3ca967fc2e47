"""Per-model entry scripts (reference <model>/cifar10_<model>_<mode>.py, imagenet_inception_<mode>.py
and the eval scripts).  Run as ``python -m distributed_tensorflow_models_amd.trainers.<name>``."""
