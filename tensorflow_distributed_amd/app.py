"""``tf.app`` analogue: ``app.flags`` (absl/gflags-style definitions) and ``app.run(main)``.

Reference usage: ``flags = tf.app.flags; FLAGS = flags.FLAGS; ... tf.app.run()``
(``/root/reference/mnist_python_m.py:49-87, 323-324``).
"""
from .utils import flags  # noqa: F401
from .utils.flags import FLAGS, run  # noqa: F401
