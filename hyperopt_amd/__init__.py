"""hyperopt_amd — MI355X-native Tree-structured Parzen Estimator suggest path.

Drop-in for the TPE path of gsmafra/hyperopt 0.0.3 (``hyperopt/__init__.py``):
the same ``hp``, ``fmin``, ``tpe.suggest``, ``rand.suggest``, ``Trials``,
``Domain`` and constants.  The O(C x K) candidate scoring runs in HIP kernels
for gfx950 (``libtpe_hip.so``, C-ABI in include/tpe_hip.h); there is no CPU
fallback for it.
"""
from . import hp  # noqa: F401
from . import exceptions  # noqa: F401
from . import rand  # noqa: F401
from . import tpe  # noqa: F401
from .base import (STATUS_STRINGS, STATUS_NEW, STATUS_OK, STATUS_FAIL, JOB_STATES,  # noqa: F401
                   JOB_STATE_NEW, JOB_STATE_RUNNING, JOB_STATE_DONE, JOB_STATE_ERROR,
                   Ctrl, Trials, Domain)
from .fmin import fmin, fmin_path, FMinIter  # noqa: F401
from .space import scope  # noqa: F401

__version__ = '0.1.0'
