"""Reference ``bigdl.util.engine`` (P/util/engine.py): environment preparation for a BigDL job.

The reference locates Spark (pyspark or SPARK_HOME), the BigDL jar and its conf file and puts them on the paths.
Here there is no JVM: ``prepare_env`` only honours ``BIGDL_PACKAGES`` (extra Python paths) and the version /
classpath helpers keep their reference behaviour so launch scripts that call them keep working."""
import os
import sys
import warnings


def exist_pyspark():
    try:
        import pyspark  # noqa: F401
        return True
    except ImportError:
        return False


def check_spark_source_conflict(spark_home, pyspark_path):
    """Warn when SPARK_HOME and the imported pyspark point at different installations."""
    if spark_home and not pyspark_path.startswith(spark_home):
        warnings.warn(f"SPARK_HOME is {spark_home} but pyspark was found in {pyspark_path}; use one of them")


def get_bigdl_classpath():
    """BIGDL_CLASSPATH if set, else "" (the engine ships no jar)."""
    return os.environ.get("BIGDL_CLASSPATH", "")


def compare_version(version1, version2):
    """1 / -1 / 0 as version1 is after / before / equal to version2 (missing components count as 0)."""
    a = [int(t) for t in version1.split(".")]
    b = [int(t) for t in version2.split(".")]
    n = max(len(a), len(b))
    a, b = a + [0] * (n - len(a)), b + [0] * (n - len(b))
    return (a > b) - (a < b)


def is_spark_below_2_2():
    """True when an installed pyspark is older than 2.2; False without pyspark (no SPARK_CLASSPATH needed)."""
    if not exist_pyspark():
        return False
    import pyspark

    ver = getattr(getattr(pyspark, "version", None), "__version__", None)
    if ver is None:
        return True
    major_minor = ".".join(ver.split(".")[:2])
    return compare_version(major_minor, "2.2") < 0


def prepare_env():
    """Prepend every BIGDL_PACKAGES entry (':'-separated) to sys.path."""
    for package in filter(None, os.environ.get("BIGDL_PACKAGES", "").split(":")):
        if package not in sys.path:
            sys.path.insert(0, package)


__all__ = ["exist_pyspark", "check_spark_source_conflict", "get_bigdl_classpath", "compare_version",
           "is_spark_below_2_2", "prepare_env"]
