"""Model save / load in Spark's on-disk formats (host side; pyarrow).

Mirrors the writers and readers a Spark user's pipeline relies on, so a model
trained here loads in Spark (and back):
  - mllib KMeansModel, format "2.0" (mllib/clustering/KMeansModel.scala:
    148-224, SaveLoadV2_0): metadata/part-00000 = one JSON line
    {"class", "version", "k", "distanceMeasure", "trainingCost"};
    data/ = parquet rows Cluster(id: Int, point: mllib Vector);
  - ml LogisticRegressionModel (ml/classification/LogisticRegression.scala:
    1304-1360): metadata/part-00000 = DefaultParamsWriter.getMetadataToSave
    (ml/util/ReadWrite.scala:422-451: class, timestamp, sparkVersion, uid,
    paramMap, defaultParamMap); data/ = one parquet row Data(numClasses,
    numFeatures, interceptVector: ml Vector, coefficientMatrix: Matrix,
    isMultinomial).
Vectors and matrices use the UDT struct encodings (ml/linalg/VectorUDT.scala,
MatrixUDT.scala:30-70, mllib/linalg/Vectors.scala:271-280): type 1 = dense
(values; matrices also numRows/numCols/isTransposed), type 0 = sparse.
Spark recovers the UDTs from the Spark row schema it stores in the parquet
footer under "org.apache.spark.sql.parquet.row.metadata"; the writers here
store the same JSON.  The readers accept both encodings of either UDT, as
Spark itself writes them (checked against the reference's own saved-model
fixture, tests/golden/ml-models/mlp-2.4.4).
"""
from __future__ import annotations

import json
import os
import time
import uuid

import numpy as np

SPARK_VERSION = "3.3.0"
ROW_META = b"org.apache.spark.sql.parquet.row.metadata"


def _pa():
    import pyarrow as pa
    import pyarrow.parquet as pq
    return pa, pq


# -- UDT encodings -------------------------------------------------------------

def _vector_sqltype():
    return {"type": "struct", "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "size", "type": "integer", "nullable": True, "metadata": {}},
        {"name": "indices", "type": {"type": "array", "elementType": "integer",
                                     "containsNull": False}, "nullable": True, "metadata": {}},
        {"name": "values", "type": {"type": "array", "elementType": "double",
                                    "containsNull": False}, "nullable": True, "metadata": {}}]}


def _matrix_sqltype():
    arr = lambda t: {"type": "array", "elementType": t, "containsNull": False}
    return {"type": "struct", "fields": [
        {"name": "type", "type": "byte", "nullable": False, "metadata": {}},
        {"name": "numRows", "type": "integer", "nullable": False, "metadata": {}},
        {"name": "numCols", "type": "integer", "nullable": False, "metadata": {}},
        {"name": "colPtrs", "type": arr("integer"), "nullable": True, "metadata": {}},
        {"name": "rowIndices", "type": arr("integer"), "nullable": True, "metadata": {}},
        {"name": "values", "type": arr("double"), "nullable": True, "metadata": {}},
        {"name": "isTransposed", "type": "boolean", "nullable": False, "metadata": {}}]}


def _udt(kind, ml=True):
    pkg = "ml" if ml else "mllib"
    cls = "VectorUDT" if kind == "vector" else "MatrixUDT"
    return {"type": "udt", "class": f"org.apache.spark.{pkg}.linalg.{cls}",
            "pyClass": f"pyspark.{pkg}.linalg.{cls}",
            "sqlType": _vector_sqltype() if kind == "vector" else _matrix_sqltype()}


def _arrow_vector():
    pa, _ = _pa()
    return pa.struct([pa.field("type", pa.int8(), nullable=False),
                      pa.field("size", pa.int32()),
                      pa.field("indices", pa.list_(pa.field("element", pa.int32(), nullable=False))),
                      pa.field("values", pa.list_(pa.field("element", pa.float64(),
                                                           nullable=False)))])


def _arrow_matrix():
    pa, _ = _pa()
    li = lambda t: pa.list_(pa.field("element", t, nullable=False))
    return pa.struct([pa.field("type", pa.int8(), nullable=False),
                      pa.field("numRows", pa.int32(), nullable=False),
                      pa.field("numCols", pa.int32(), nullable=False),
                      pa.field("colPtrs", li(pa.int32())),
                      pa.field("rowIndices", li(pa.int32())),
                      pa.field("values", li(pa.float64())),
                      pa.field("isTransposed", pa.bool_(), nullable=False)])


def encode_dense_vector(v):
    """VectorUDT.serialize of a DenseVector."""
    return {"type": 1, "size": None, "indices": None,
            "values": [float(x) for x in np.asarray(v, dtype=np.float64).ravel()]}


def decode_vector(d) -> np.ndarray:
    """VectorUDT.deserialize (either encoding) to a dense numpy vector."""
    if d["type"] == 1:
        return np.asarray(d["values"], dtype=np.float64)
    if d["type"] != 0:
        raise ValueError(f"unknown vector type {d['type']}")
    out = np.zeros(int(d["size"]))
    out[np.asarray(d["indices"], dtype=np.int64)] = np.asarray(d["values"], dtype=np.float64)
    return out


def encode_dense_matrix(M, isTransposed=True):
    """MatrixUDT.serialize of DenseMatrix(numRows, numCols, values,
    isTransposed): values row-major when transposed, else column-major."""
    M = np.asarray(M, dtype=np.float64)
    vals = M.ravel(order="C" if isTransposed else "F")
    return {"type": 1, "numRows": int(M.shape[0]), "numCols": int(M.shape[1]), "colPtrs": None,
            "rowIndices": None, "values": [float(x) for x in vals],
            "isTransposed": bool(isTransposed)}


def decode_matrix(d) -> np.ndarray:
    """MatrixUDT.deserialize (dense or sparse, transposed or not)."""
    r, c = int(d["numRows"]), int(d["numCols"])
    vals = np.asarray(d["values"], dtype=np.float64)
    if d["type"] == 1:
        return vals.reshape(r, c) if d["isTransposed"] else vals.reshape(c, r).T.copy()
    if d["type"] != 0:
        raise ValueError(f"unknown matrix type {d['type']}")
    ptr = np.asarray(d["colPtrs"], dtype=np.int64)
    idx = np.asarray(d["rowIndices"], dtype=np.int64)
    out = np.zeros((r, c))
    if d["isTransposed"]:     # CSR: colPtrs index rows, rowIndices hold columns
        for i in range(r):
            out[i, idx[ptr[i]:ptr[i + 1]]] = vals[ptr[i]:ptr[i + 1]]
    else:
        for j in range(c):
            out[idx[ptr[j]:ptr[j + 1]], j] = vals[ptr[j]:ptr[j + 1]]
    return out


# -- files ---------------------------------------------------------------------

def _write_text(dirpath, line):
    os.makedirs(dirpath, exist_ok=False)
    with open(os.path.join(dirpath, "part-00000"), "w") as f:
        f.write(line + "\n")
    open(os.path.join(dirpath, "_SUCCESS"), "w").close()


def _read_text(dirpath):
    parts = sorted(p for p in os.listdir(dirpath) if p.startswith("part-"))
    for p in parts:
        with open(os.path.join(dirpath, p)) as f:
            for line in f:
                if line.strip():
                    return line.strip()
    raise FileNotFoundError(f"no metadata line under {dirpath}")


def _write_parquet(dirpath, schema_fields, spark_fields, rows):
    """One part file + _SUCCESS, with Spark's row schema in the footer."""
    pa, pq = _pa()
    os.makedirs(dirpath, exist_ok=False)
    spark_schema = json.dumps({"type": "struct", "fields": spark_fields}, separators=(",", ":"))
    schema = pa.schema(schema_fields, metadata={ROW_META: spark_schema.encode()})
    cols = {f.name: [r[f.name] for r in rows] for f in schema_fields}
    table = pa.Table.from_pydict(cols, schema=schema)
    name = f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"
    pq.write_table(table, os.path.join(dirpath, name), compression="snappy")
    open(os.path.join(dirpath, "_SUCCESS"), "w").close()


def _read_parquet_rows(dirpath):
    _, pq = _pa()
    rows = []
    for p in sorted(os.listdir(dirpath)):
        if p.endswith(".parquet"):
            rows.extend(pq.read_table(os.path.join(dirpath, p)).to_pylist())
    return rows


def _field(name, typ, nullable=True):
    return {"name": name, "type": typ, "nullable": nullable, "metadata": {}}


def _check_new_path(path, overwrite):
    if os.path.exists(path):
        if not overwrite:
            raise IOError(f"Path {path} already exists. To overwrite it, please use "
                          "write.overwrite().save(path) for Scala and use "
                          "write().overwrite().save(path) for Java and Python.")
        import shutil
        shutil.rmtree(path)


# -- mllib KMeansModel ---------------------------------------------------------

KMEANS_CLASS = "org.apache.spark.mllib.clustering.KMeansModel"


def save_kmeans_model(model, path, distanceMeasure="euclidean", overwrite=False,
                      version="2.0"):
    """KMeansModel.SaveLoadV2_0.save (KMeansModel.scala:195-206); version
    "1.0" writes SaveLoadV1_0's layout (:162-171: metadata without
    distanceMeasure / trainingCost), the format of older Spark releases."""
    pa, _ = _pa()
    _check_new_path(path, overwrite)
    if version == "1.0":
        meta = json.dumps({"class": KMEANS_CLASS, "version": "1.0", "k": int(model.k)},
                          separators=(",", ":"))
    elif version == "2.0":
        meta = json.dumps({"class": KMEANS_CLASS, "version": "2.0", "k": int(model.k),
                           "distanceMeasure": distanceMeasure,
                           "trainingCost": float(model.trainingCost)}, separators=(",", ":"))
    else:
        raise ValueError(f"unsupported KMeansModel format version {version}")
    _write_text(os.path.join(path, "metadata"), meta)
    fields = [pa.field("id", pa.int32(), nullable=False), pa.field("point", _arrow_vector())]
    spark = [_field("id", "integer", False), _field("point", _udt("vector", ml=False))]
    rows = [{"id": i, "point": encode_dense_vector(c)} for i, c in enumerate(model.clusterCenters)]
    _write_parquet(os.path.join(path, "data"), fields, spark, rows)


def load_kmeans_model(path):
    """KMeansModel.load (KMeansModel.scala:130-145): SaveLoadV2_0.load
    (:208-222) -- centers sorted by id, trainingCost and distanceMeasure from
    the metadata -- or SaveLoadV1_0.load (:173-185), whose model is
    `new KMeansModel(centers)`: Euclidean, trainingCost 0.0.  numIter is
    unknown (-1 in the reference) either way."""
    from .clustering import KMeansModel
    meta = json.loads(_read_text(os.path.join(path, "metadata")))
    version = meta.get("version")
    if meta.get("class") != KMEANS_CLASS or version not in ("1.0", "2.0"):
        raise ValueError(f"KMeansModel.load did not recognize model with (className, format "
                         f"version):({meta.get('class')}, {version}).  Supported:\n"
                         f"  ({KMEANS_CLASS}, 1.0)\n  ({KMEANS_CLASS}, 2.0)")
    if version == "1.0":
        meta = {"k": meta["k"]}             # V1 defaults below: euclidean, cost 0.0
    rows = _read_parquet_rows(os.path.join(path, "data"))
    if len(rows) != int(meta["k"]):
        raise ValueError(f"expected {meta['k']} centers, found {len(rows)}")
    rows.sort(key=lambda r: r["id"])
    C = np.stack([decode_vector(r["point"]) for r in rows])
    return KMeansModel(C, trainingCost=float(meta.get("trainingCost", 0.0)), numIter=-1,
                       distanceMeasure=meta.get("distanceMeasure", "euclidean"))


# -- ml LogisticRegressionModel -----------------------------------------------

LR_CLASS = "org.apache.spark.ml.classification.LogisticRegressionModel"


def _lr_params(est):
    """paramMap as copyValues(estimator) leaves it on the model."""
    p = {"featuresCol": "features", "labelCol": "label", "predictionCol": "prediction",
         "rawPredictionCol": "rawPrediction", "probabilityCol": "probability"}
    if est is not None:
        p.update({"regParam": est.regParam, "elasticNetParam": est.elasticNetParam,
                  "maxIter": est.maxIter, "tol": est.tol, "fitIntercept": est.fitIntercept,
                  "standardization": est.standardization, "family": est.family,
                  "aggregationDepth": est.aggregationDepth,
                  "maxBlockSizeInMB": est.maxBlockSizeInMB})
    return p


_LR_DEFAULTS = {"regParam": 0.0, "elasticNetParam": 0.0, "maxIter": 100, "tol": 1e-6,
                "fitIntercept": True, "standardization": True, "family": "auto",
                "threshold": 0.5, "aggregationDepth": 2, "maxBlockSizeInMB": 0.0,
                "featuresCol": "features", "labelCol": "label", "predictionCol": "prediction",
                "rawPredictionCol": "rawPrediction", "probabilityCol": "probability"}


def save_logistic_model(model, path, estimator=None, uid=None, overwrite=False):
    """LogisticRegressionModelWriter.saveImpl (LogisticRegression.scala:1314-1322)."""
    pa, _ = _pa()
    _check_new_path(path, overwrite)
    params = _lr_params(estimator)
    if estimator is None and not getattr(model, "fitIntercept", True):
        params["fitIntercept"] = False          # the model's own param, when set
    meta = {"class": LR_CLASS, "timestamp": int(time.time() * 1000),
            "sparkVersion": SPARK_VERSION,
            "uid": uid or f"logreg_{uuid.uuid4().hex[:12]}",
            "paramMap": params, "defaultParamMap": dict(_LR_DEFAULTS)}
    _write_text(os.path.join(path, "metadata"), json.dumps(meta, separators=(",", ":")))
    fields = [pa.field("numClasses", pa.int32(), nullable=False),
              pa.field("numFeatures", pa.int32(), nullable=False),
              pa.field("interceptVector", _arrow_vector()),
              pa.field("coefficientMatrix", _arrow_matrix()),
              pa.field("isMultinomial", pa.bool_(), nullable=False)]
    spark = [_field("numClasses", "integer", False), _field("numFeatures", "integer", False),
             _field("interceptVector", _udt("vector")), _field("coefficientMatrix",
                                                               _udt("matrix")),
             _field("isMultinomial", "boolean", False)]
    row = {"numClasses": int(model.numClasses), "numFeatures": int(model.numFeatures),
           "interceptVector": encode_dense_vector(model.interceptVector),
           "coefficientMatrix": encode_dense_matrix(model.coefficientMatrix, True),
           "isMultinomial": bool(model.isMultinomial)}
    _write_parquet(os.path.join(path, "data"), fields, spark, [row])


def load_logistic_model(path):
    """LogisticRegressionModelReader.load (:1330-1360), Spark >= 2.1 data."""
    from .classification import LogisticRegressionModel
    meta = json.loads(_read_text(os.path.join(path, "metadata")))
    if meta.get("class") != LR_CLASS:
        raise ValueError(f"requirement failed: Error loading metadata: Expected class name "
                         f"{LR_CLASS} but found class name {meta.get('class')}")
    major, minor = (int(x) for x in meta["sparkVersion"].split(".")[:2])
    rows = _read_parquet_rows(os.path.join(path, "data"))
    if len(rows) != 1:
        raise ValueError("expected one data row")
    r = rows[0]
    if major < 2 or (major == 2 and minor == 0):
        # 2.0 and earlier: numClasses, numFeatures, intercept, coefficients (binomial only)
        coef = decode_vector(r["coefficients"]).reshape(1, -1)
        icpt = np.array([float(r["intercept"])])
        return LogisticRegressionModel(coef, icpt, int(r["numClasses"]), False)
    m = LogisticRegressionModel(decode_matrix(r["coefficientMatrix"]),
                                decode_vector(r["interceptVector"]), int(r["numClasses"]),
                                bool(r["isMultinomial"]))
    m.uid = meta.get("uid")
    m.params = dict(meta.get("defaultParamMap", {}), **meta.get("paramMap", {}))
    m.fitIntercept = bool(m.params.get("fitIntercept", True))
    return m


def read_metadata(path):
    """DefaultParamsReader.loadMetadata (ReadWrite.scala:585-615) -> dict."""
    return json.loads(_read_text(os.path.join(path, "metadata")))
