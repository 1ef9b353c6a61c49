"""TEST INFRASTRUCTURE ONLY: the CPU oracle (see xsalsa_oracle.c).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by rclone_amd/."""
