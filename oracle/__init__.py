"""CPU oracle for NepTUN's data-path AEAD -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package, and only as the checker. neptun_amd/ never imports it.
"""
