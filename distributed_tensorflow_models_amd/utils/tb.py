"""Minimal TensorBoard event writer (tf.Event / Summary protos in TFRecord framing) so eval/train
scalars ('Precision @ 1', 'Recall @ 5', 'learning_rate', 'total_loss') land where TensorBoard reads."""
import os
import socket
import struct
import time

from ..data.tfrecord import TFRecordWriter, _ld, _varint


def _event(wall, step=None, summary=None, file_version=None):
    b = _varint((1 << 3) | 1) + struct.pack("<d", wall)
    if step is not None:
        b += _varint(2 << 3) + _varint(int(step))
    if file_version is not None:
        b += _ld(3, file_version.encode())
    if summary is not None:
        b += _ld(5, summary)
    return b


def _scalar_summary(tag, value):
    v = _ld(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
    return _ld(1, v)


class SummaryWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname())
        self.path = os.path.join(logdir, name)
        self.w = TFRecordWriter(self.path)
        self.w.write(_event(time.time(), file_version="brain.Event:2"))

    def add_scalar(self, tag, value, step):
        self.w.write(_event(time.time(), step, _scalar_summary(tag, value)))

    def close(self):
        self.w.close()
