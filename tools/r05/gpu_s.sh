#!/bin/bash
# round-5 GPU pass S: ROC_GLOBAL_CU_MASK semantics on gfx950 (which CUs / XCDs a masked launch uses)
cd "$GRAFT_REPO_ROOT" || exit 1
for m in "" 0xf 0xff 0xffffffff 0xffffffffffffffff 0xffffffff00000000 0xffffffffffffffffffffffffffffffff \
         0xffffffffffffffffffffffffffffffff00000000000000000000000000000000 \
         0x0000000000000000ffffffffffffffff; do
  if [ -z "$m" ]; then timeout -k 5 30 ./tools/probes/cu_mask_probe || exit 1
  else ROC_GLOBAL_CU_MASK=$m timeout -k 5 30 ./tools/probes/cu_mask_probe || exit 1; fi
done
