"""Entry script: reference resnet/cifar10_resnet_bsp.py (preset ``resnet``, default sync mode ``bsp``).

Accepts the reference flags (--job_name/--ps_hosts/--worker_hosts/--task_id/--batch_size/--data_dir/
--train_dir/--max_steps ...) plus the MI355X extras (--sync_mode, --synthetic_data, --fresh, ...).
"""
from ..compat import flags
from .. import trainer

trainer.define_common_flags(flags, "resnet")


def main(_argv=None):
    return trainer.train("resnet", flags, default_mode="bsp")


if __name__ == "__main__":
    flags.run(main)
