"""Does this node have the host CPUs to feed its GPUs real ImageNet?  (the reference sizes its input
by giving every worker HOST its own decode stream: /root/reference/inception/image_processing.py:476-503, one worker
per host, /root/reference/train.sh:53-61.  One MI355X node runs 8 such workers.)

Host CPU time per training image, measured on one core by tools/decode_cpu_cost.py (log: profiles/r5/
r5_decode_cpu_cost*.log):
  full  - Example parse + baseline JPEG decode (PIL / libjpeg-turbo) + distortion parameters,
  split - the same with only the Huffman decode on the host (DTM_SPLIT_DECODE=1: dequantisation, IDCT, upsampling
          and colour conversion run as HIP kernels, csrc/kernels/jpeg.hip).
The split path needs ~1.8x less host CPU per image on the box (729 vs 410 us; 2.4x on this container's slower cores,
r5_decode_cpu_cost_container.log); on a box with CPUs to spare the full path sustains more
images/s (its batch assembly is lighter: profiles/r3/r3_imagenet_pipeline_split_vs_full.log), so it stays the default
there, and ``choose_split_decode`` switches to split only when full decode cannot keep up."""
import logging
import os

# img/s per host CPU core (tools/decode_cpu_cost.py on the MI355X box's host CPUs; see module docstring)
IMG_S_PER_CPU = {"full": 1370.0, "split": 2440.0}

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


def decode_capacity_check(model, gpus=None, cpus=None, mode="full", log=None, per_cpu=None):
    """Warn when the host CPUs of this node cannot decode images as fast as its ``gpus`` ranks train on them.
    Returns (needed CPUs, available CPUs, ok)."""
    log = log or logging.getLogger("distributed_tensorflow_models_amd").warning
    gpus = local_world() if gpus is None else gpus
    cpus = node_cpus() if cpus is None else cpus
    per_gpu = PER_GPU_IMG_S.get(model)
    if per_gpu is None:
        return None, cpus, True
    need = needed_cpus(per_gpu, gpus, mode, per_cpu)
    ok = need <= cpus
    if not ok:
        other = "split" if mode == "full" else "full"
        log("input pipeline: %d rank(s) of %s consume ~%.0f img/s; %s JPEG decode needs ~%.0f host CPUs at %.0f img/s "
            "per CPU, this process may use %d - training will be input-bound (~%.0f %% of the GPU rate)%s" % (
                gpus, model, gpus * per_gpu, mode, need, (per_cpu or IMG_S_PER_CPU)[mode], cpus,
                100.0 * cpus / need,
                "; the %s decode needs ~%.0f" % (other, needed_cpus(per_gpu, gpus, other, per_cpu))))
    return need, cpus, ok


def choose_split_decode(model, gpus=None, cpus=None, per_cpu=None):
    """DTM_SPLIT_DECODE unset: the split decode when the full one cannot keep the node's GPUs fed and split can
    (or comes closer); 0 / 1 force a mode."""
    env = os.environ.get("DTM_SPLIT_DECODE")
    if env is not None:
        return env == "1"
    per_gpu = PER_GPU_IMG_S.get(model)
    if per_gpu is None:
        return False
    gpus = local_world() if gpus is None else gpus
    cpus = node_cpus() if cpus is None else cpus
    split = needed_cpus(per_gpu, gpus, "full", per_cpu) > cpus
    logging.getLogger("distributed_tensorflow_models_amd").info(
        "input pipeline: %s JPEG decode (%d rank(s) on %d CPUs, %s)", "split" if split else "full", gpus, cpus, model)
    return split
