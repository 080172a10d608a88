"""qe_hip — Python binding of the MI355X qeh backend (C ABI: include/qeh.h).

Import with the package directory on sys.path:
    sys.path.insert(0, "<repo>/query-engine_amd"); import qe_hip
"""
from . import abi  # noqa: F401
from .abi import QehError, load  # noqa: F401
from .device import Context, DeviceColumn, agg  # noqa: F401
from .expr import (AggregateExpr, AggregateFunction, BinaryExpr, BinaryOp, Column,  # noqa: F401
                   Literal, PhysicalExpr, ScalarValue, UnaryExpr, UnaryOp, binop, col, lit)
from .plan import (DataSource, Filter, HashAggregate, HashJoin, IndexScan, JoinType, Limit,  # noqa: F401
                   MemoryDataSource, Projection, QueryExecutor, Scan, Sort, SubqueryScan, Window, WindowExpr,
                   WindowFunctionType)
from .merge import Merge, MergeStrategy, SortColumn  # noqa: F401,E402
from .partition import DeviceBatch, Exchange, Partition, Partitioner, PartitionStrategy  # noqa: F401,E402
