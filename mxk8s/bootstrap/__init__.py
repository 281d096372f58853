"""Host bring-up for a single-node MI355X Kubernetes cluster (``mxk8s bootstrap``)."""
from .phases import PHASES, PHASE_NAMES, Context, PhaseError, run, completed  # noqa: F401
from . import hostfiles  # noqa: F401
