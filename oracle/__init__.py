"""ORACLE -- CPU restatements of the reference (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product path (snd_vae_amd) never does.
"""
