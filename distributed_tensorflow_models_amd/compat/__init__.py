"""TensorFlow 1.x API facades (flags, logging, tf.train, slim) over the native engine."""
