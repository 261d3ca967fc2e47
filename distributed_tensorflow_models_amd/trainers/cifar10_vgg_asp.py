"""Entry script: reference vgg/cifar10_vgg_asp.py (preset ``vgg_asp``, default sync mode ``asp``).

Accepts the reference flags (--job_name/--ps_hosts/--worker_hosts/--task_id/--batch_size/--data_dir/
--train_dir/--max_steps ...) plus the MI355X extras (--sync_mode, --synthetic_data, --fresh, ...).
"""
from ..compat import flags
from .. import trainer

trainer.define_common_flags(flags, "vgg_asp")


def main(_argv=None):
    return trainer.train("vgg_asp", flags, default_mode="asp")


if __name__ == "__main__":
    flags.run(main)
