"""ORACLE — CPU restatement of the reference's hot path, used ONLY as the checker
(tests/, __graft_entry__.smoke()) and as bench.py's timed cpu_baseline.  Never
imported by the product package (book-recommendation-engine_amd/vsearch)."""
