"""Entry script: reference cnn/cifar10_cnn_bsp.py (preset ``cnn``, default sync mode ``bsp``).

Accepts the reference flags (--job_name/--ps_hosts/--worker_hosts/--task_id/--batch_size/--data_dir/
--train_dir/--max_steps ...) plus the MI355X extras (--sync_mode, --synthetic_data, --fresh, ...).
"""
from ..compat import flags
from .. import trainer

trainer.define_common_flags(flags, "cnn")


def main(_argv=None):
    return trainer.train("cnn", flags, default_mode="bsp")


if __name__ == "__main__":
    flags.run(main)
