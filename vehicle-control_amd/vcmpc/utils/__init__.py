from .fancy_vector import FancyVector  # noqa: F401
from .common_utils import wrap  # noqa: F401
