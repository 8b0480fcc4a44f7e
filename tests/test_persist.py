"""Model save / load in Spark's formats (cycloneml_amd.persist).

The UDT encodings and the footer schema are checked against a model Spark
itself wrote: the reference's MultilayerPerceptronClassificationModel fixture
(mllib/src/test/resources/ml-models/mlp-2.4.4, copied to tests/golden as
data), whose `weights` column is an ml VectorUDT.  Round trips cover the
mllib KMeansModel format 2.0 (KMeansModel.scala:189-223) and the ml
LogisticRegressionModel writer / reader (LogisticRegression.scala:1304-1360),
binomial and multinomial, including the sparse matrix encoding Spark uses
for compressed coefficient matrices."""
import json
import os

import numpy as np
import pytest

from cycloneml_amd import persist
from cycloneml_amd.classification import LogisticRegression, LogisticRegressionModel
from cycloneml_amd.clustering import KMeansModel

FIX = os.path.join(os.path.dirname(__file__), "golden", "ml-models", "mlp-2.4.4")


def _spark_schema(dirpath):
    import pyarrow.parquet as pq
    f = [p for p in os.listdir(dirpath) if p.endswith(".parquet")][0]
    md = pq.read_schema(os.path.join(dirpath, f)).metadata
    return json.loads(md[persist.ROW_META])


def test_reads_spark_written_vector_udt():
    meta = persist.read_metadata(FIX)
    assert meta["class"] == "org.apache.spark.ml.classification.MultilayerPerceptronClassificationModel"
    assert meta["sparkVersion"] == "2.4.4"
    rows = persist._read_parquet_rows(os.path.join(FIX, "data"))
    assert rows[0]["layers"] == [4, 5, 2]
    w = persist.decode_vector(rows[0]["weights"])
    # layers 4-5-2: (4 + 1) * 5 + (5 + 1) * 2 weights
    assert w.shape == (37,)
    assert w[0] == 0.562493954827742 and w[1] == -2.921111622795348


def test_vector_udt_footer_matches_spark():
    """The sqlType this writer stores equals the one Spark stored."""
    spark = _spark_schema(os.path.join(FIX, "data"))
    wfield = [f for f in spark["fields"] if f["name"] == "weights"][0]["type"]
    assert wfield["class"] == "org.apache.spark.ml.linalg.VectorUDT"
    assert wfield["sqlType"] == persist._vector_sqltype()
    assert persist._udt("vector") == {k: wfield[k] for k in ("type", "class", "pyClass",
                                                              "sqlType")}


def test_kmeans_model_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    m = KMeansModel(rng.normal(size=(7, 5)), trainingCost=12.5, numIter=9)
    p = str(tmp_path / "km")
    m.save(p)
    meta = persist.read_metadata(p)
    assert meta == {"class": "org.apache.spark.mllib.clustering.KMeansModel", "version": "2.0",
                    "k": 7, "distanceMeasure": "euclidean", "trainingCost": 12.5}
    sch = _spark_schema(os.path.join(p, "data"))
    assert [f["name"] for f in sch["fields"]] == ["id", "point"]
    assert sch["fields"][1]["type"]["class"] == "org.apache.spark.mllib.linalg.VectorUDT"
    m2 = KMeansModel.load(p)
    assert np.array_equal(m2.clusterCenters, m.clusterCenters)
    assert m2.trainingCost == 12.5 and m2.numIter == -1
    with pytest.raises(IOError, match="already exists"):
        m.save(p)
    m.save(p, overwrite=True)


@pytest.mark.parametrize("multinomial", [False, True])
def test_logistic_model_round_trip(tmp_path, multinomial):
    rng = np.random.default_rng(1)
    C = 3 if multinomial else 1
    m = LogisticRegressionModel(rng.normal(size=(C, 6)), rng.normal(size=C),
                                3 if multinomial else 2, multinomial)
    p = str(tmp_path / "lr")
    est = LogisticRegression(regParam=0.1, elasticNetParam=0.5, maxIter=50)
    m.save(p, estimator=est)
    meta = persist.read_metadata(p)
    assert meta["class"] == "org.apache.spark.ml.classification.LogisticRegressionModel"
    assert meta["paramMap"]["regParam"] == 0.1 and meta["paramMap"]["maxIter"] == 50
    assert meta["defaultParamMap"]["tol"] == 1e-6
    sch = _spark_schema(os.path.join(p, "data"))
    names = [f["name"] for f in sch["fields"]]
    assert names == ["numClasses", "numFeatures", "interceptVector", "coefficientMatrix",
                     "isMultinomial"]
    assert sch["fields"][3]["type"]["class"] == "org.apache.spark.ml.linalg.MatrixUDT"
    m2 = LogisticRegressionModel.load(p)
    assert np.array_equal(m2.coefficientMatrix, m.coefficientMatrix)
    assert np.array_equal(m2.interceptVector, m.interceptVector)
    assert m2.numClasses == m.numClasses and m2.isMultinomial == multinomial
    assert m2.params["elasticNetParam"] == 0.5


def test_matrix_udt_sparse_and_column_major():
    M = np.array([[0.0, 1.5, 0.0], [2.0, 0.0, -3.0]])
    # column-major dense
    d = persist.encode_dense_matrix(M, isTransposed=False)
    assert np.array_equal(persist.decode_matrix(d), M)
    # SparseMatrix CSC (isTransposed = false) and CSR (true), as Spark encodes them
    csc = {"type": 0, "numRows": 2, "numCols": 3, "colPtrs": [0, 1, 2, 3],
           "rowIndices": [1, 0, 1], "values": [2.0, 1.5, -3.0], "isTransposed": False}
    csr = {"type": 0, "numRows": 2, "numCols": 3, "colPtrs": [0, 1, 3],
           "rowIndices": [1, 0, 2], "values": [1.5, 2.0, -3.0], "isTransposed": True}
    assert np.array_equal(persist.decode_matrix(csc), M)
    assert np.array_equal(persist.decode_matrix(csr), M)
    sv = {"type": 0, "size": 5, "indices": [1, 4], "values": [2.0, -1.0], }
    assert np.array_equal(persist.decode_vector(sv), [0.0, 2.0, 0.0, 0.0, -1.0])


def test_wrong_class_is_refused(tmp_path):
    p = str(tmp_path / "km")
    KMeansModel(np.zeros((2, 2))).save(p)
    with pytest.raises(ValueError, match="Expected class name"):
        LogisticRegressionModel.load(p)


def test_kmeans_model_v1_format(tmp_path):
    """KMeansModel.load of SaveLoadV1_0's layout (KMeansModel.scala:156-186:
    metadata {class, version 1.0, k} only): `new KMeansModel(centers)`, so
    Euclidean with trainingCost 0.0; an unknown version is refused with the
    reference's message."""
    rng = np.random.default_rng(1)
    C = rng.normal(size=(4, 3))
    p = str(tmp_path / "km1")
    persist.save_kmeans_model(KMeansModel(C, trainingCost=3.0), p, version="1.0")
    assert persist.read_metadata(p) == {"class": "org.apache.spark.mllib.clustering.KMeansModel",
                                        "version": "1.0", "k": 4}
    m = KMeansModel.load(p)
    assert np.array_equal(m.clusterCenters, C)
    assert m.trainingCost == 0.0 and m.numIter == -1 and m.distanceMeasure == "euclidean"
    meta = os.path.join(p, "metadata")
    for f in os.listdir(meta):
        if f.startswith("part-"):
            txt = open(os.path.join(meta, f)).read().replace('"1.0"', '"3.0"')
            open(os.path.join(meta, f), "w").write(txt)
    with pytest.raises(ValueError, match="did not recognize model"):
        KMeansModel.load(p)
