"""MI355X-native distributed CNN training framework.

A from-scratch re-design (not a port) of the capabilities of
``chenc10/distributed_TensorFlow_models`` for AMD Instinct MI355X (gfx950):

* ``ops``       - hand-written CDNA4 HIP kernels (implicit-GEMM conv, fused BatchNorm, pooling,
                  softmax cross-entropy, multi-tensor optimizers) behind autograd Functions.
* ``models``    - the reference model zoo with TF variable names (``nets_factory``).
* ``parallel``  - BSP bucketed all-reduce over RCCL/xGMI, ASP owner-sharded parameter store,
                  SSP staleness clock, launcher.
* ``compat``    - thin ``tf.app.flags`` / ``tf.train`` / ``slim`` facade.
* ``ckpt``      - TensorFlow TensorBundle checkpoints (native C++ reader/writer).
* ``data``      - synthetic ImageNet/CIFAR/MNIST, CIFAR-binary and TFRecord readers, augmentation.
* ``eval``      - polling evaluators (precision@1, recall@5, EMA restore).
* ``utils``     - step timers, JSONL metrics, profiler hooks, TensorBoard event writer.
"""
__version__ = "0.1.0"
