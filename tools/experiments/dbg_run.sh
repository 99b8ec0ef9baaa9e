#!/bin/bash
# k-means diagnostics: ambiguous / tie / overflow counts per iteration + parity vs the oracle
ST_DEBUG=1 python tools/experiments/dbg_kmeans.py > gpurun_out/dbg.log 2>&1
