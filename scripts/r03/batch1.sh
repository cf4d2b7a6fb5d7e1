#!/bin/bash
set -u
bash scripts/r03/short.sh || exit $?
bash scripts/r03/parity_ab.sh
