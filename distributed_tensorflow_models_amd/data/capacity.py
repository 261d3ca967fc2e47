"""Does this node have the host CPUs to feed its GPUs real ImageNet?  (the reference sizes its input
by giving every worker HOST its own decode stream: /root/reference/inception/image_processing.py:476-503, one worker
per host, /root/reference/train.sh:53-61.  One MI355X node runs 8 such workers.)

Host CPU time per training image, measured on one core by tools/decode_cpu_cost.py (logs: profiles/r5/
r5_decode_cpu_cost*.log, profiles/r6/r6_decode_cpu_cost_box.log):
  full   - Example parse + baseline JPEG decode (PIL / libjpeg-turbo) + distortion parameters,
  split  - the same with only the Huffman decode on the host (DTM_SPLIT_DECODE=1: dequantisation, IDCT, upsampling
           and colour conversion run as HIP kernels, csrc/kernels/jpeg.hip),
  device - only the marker parse + byte unstuffing on the host (DTM_SPLIT_DECODE=2: the Huffman decode runs on the GPU
           too, jpeg_huff_kernel): ~10x less host CPU than split.
The full path costs the GPU nothing, so it stays the default where the CPUs keep up; ``choose_split_decode`` switches
to the device decode when they cannot (it costs the training step a few % of GPU time: profiles/r6/
r6_decode_overlap*.log)."""
import logging
import os

# img/s per host CPU core (tools/decode_cpu_cost.py on the MI355X box's host CPUs; see module docstring)
IMG_S_PER_CPU = {"full": 1370.0, "split": 2440.0, "device": 29000.0}

# expected per-GPU consumption of the training step (bench.py on one MI355X, round 5), images/s
PER_GPU_IMG_S = {"resnet_v1_50": 15000.0, "inception_v3_slim_old": 7400.0, "mobilenet_v1": 20000.0,
                 "vgg_16": 3500.0, "resnet_v1_101": 9000.0, "resnet_v1_152": 6400.0}


def node_cpus():
    """CPUs this process may run on (affinity mask; cgroup quotas are not visible here)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # (not Linux)
        return os.cpu_count() or 1


def local_world():
    """Ranks that share this process's CPUs.  When the affinity mask is narrower than the host (ranks pinned to CPU
    subsets) every rank decodes on its own CPUs: 1.  Otherwise the ranks of this node (LOCAL_WORLD_SIZE; never the
    global WORLD_SIZE, which counts other nodes' ranks)."""
    try:
        pinned = len(os.sched_getaffinity(0)) < (os.cpu_count() or 1)
    except AttributeError:
        pinned = False
    if pinned:
        return 1
    return int(os.environ.get("LOCAL_WORLD_SIZE", "1"))


def needed_cpus(per_gpu_img_s, gpus, mode="full", per_cpu=None):
    rate = (per_cpu or IMG_S_PER_CPU)[mode]
    return gpus * per_gpu_img_s / rate


MODES = ("full", "split", "device")  # DTM_SPLIT_DECODE / GPUBatchInputs split_decode = 0 / 1 / 2


def decode_capacity_check(model, gpus=None, cpus=None, mode="full", log=None, per_cpu=None):
    """Warn when the host CPUs of this node cannot decode images as fast as its ``gpus`` ranks train on them.
    ``mode``: a name of MODES or its index.  Returns (needed CPUs, available CPUs, ok)."""
    log = log or logging.getLogger("distributed_tensorflow_models_amd").warning
    mode = MODES[mode] if isinstance(mode, int) else mode
    gpus = local_world() if gpus is None else gpus
    cpus = node_cpus() if cpus is None else cpus
    per_gpu = PER_GPU_IMG_S.get(model)
    if per_gpu is None:
        return None, cpus, True
    need = needed_cpus(per_gpu, gpus, mode, per_cpu)
    ok = need <= cpus
    if not ok:
        others = "; ".join("%s decode needs ~%.0f" % (m, needed_cpus(per_gpu, gpus, m, per_cpu)) for m in MODES
                           if m != mode)
        log("input pipeline: %d rank(s) of %s consume ~%.0f img/s; %s JPEG decode needs ~%.0f host CPUs at %.0f img/s "
            "per CPU, this process may use %d - training will be input-bound (~%.0f %% of the GPU rate); %s" % (
                gpus, model, gpus * per_gpu, mode, need, (per_cpu or IMG_S_PER_CPU)[mode], cpus,
                100.0 * cpus / need, others))
    return need, cpus, ok


def choose_split_decode(model, gpus=None, cpus=None, per_cpu=None):
    """JPEG decode mode for GPUBatchInputs (0 full host decode, 1 split, 2 device decode).  DTM_SPLIT_DECODE=0/1/2
    forces one; unset: the full host decode when the node's CPUs keep its GPUs fed, else the device decode (the least
    host CPU per image)."""
    env = os.environ.get("DTM_SPLIT_DECODE")
    if env is not None:
        return {"1": 1, "2": 2, "device": 2, "split": 1}.get(env, 0)
    per_gpu = PER_GPU_IMG_S.get(model)
    if per_gpu is None:
        return 0
    gpus = local_world() if gpus is None else gpus
    cpus = node_cpus() if cpus is None else cpus
    mode = 2 if needed_cpus(per_gpu, gpus, "full", per_cpu) > cpus else 0
    logging.getLogger("distributed_tensorflow_models_amd").info(
        "input pipeline: %s JPEG decode (%d rank(s) on %d CPUs, %s)", MODES[mode], gpus, cpus, model)
    return mode
