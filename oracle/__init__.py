"""CPU oracle — TEST INFRASTRUCTURE ONLY (checker, never the product).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product path (cat-seg_amd/cat_seg) never imports it and fails
loudly when its HIP library is missing.
"""
