#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/debug_stages.py am 5 > gpurun_out/dbg.log 2>&1
