"""CPU oracle package — TEST INFRASTRUCTURE ONLY (see flat_knn.py header).

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Nothing under duckdb-lancedb_amd/ imports it.
"""
