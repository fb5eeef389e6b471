"""isim — MI355X-native simulator of isotope service-graph request traces.

Host-side mirror of isotope's graph and handler API over libisim.so
(include/isim.h).  See DESIGN.md.
"""
from .graph import (ConcurrentCommand, GraphError, RequestCommand, Service, ServiceGraph,  # noqa: F401
                    SleepCommand, duration_parse, percentage_from_string, size_from_string)
from .native import ECOMM, MODE_A, MODE_B, IsimError  # noqa: F401
from .sim import REC_DTYPE, Handler, SimParams, decode_stats, handler_from_service_graph_yaml  # noqa: F401
from .yamljson import yaml_to_json  # noqa: F401
from . import prometheus  # noqa: F401
from .des import DesHandler  # noqa: F401
