#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/soak_step.py
