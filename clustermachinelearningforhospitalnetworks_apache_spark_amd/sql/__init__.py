"""pyspark.sql-compatible front end on a sharded, device-resident columnar frame."""
from . import functions, types
from .column import Column
from .dataframe import DataFrame, DataFrameNaFunctions
from .dataframe_more import DataFrameWriterV2, Observation
from .group import GroupedData
from .session import SparkSession, Session
from .types import Row
from .window import Window, WindowSpec

__all__ = ["SparkSession", "Session", "DataFrame", "DataFrameNaFunctions", "Column", "Row", "GroupedData",
           "functions", "types", "Window", "WindowSpec"]
