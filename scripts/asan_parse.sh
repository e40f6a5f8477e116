# build the reference front end (and, with a second argument "oracle", the oracle)
# with AddressSanitizer into /tmp and run a file of SQL lines through parse +
# releaseNode (+ orc_evaluate):  bash scripts/asan_parse.sh queries.sql [oracle]
set -e
REF=${REF:-/root/reference}
OUT=/tmp/cq_asan_parse
mkdir -p $OUT
SRC="$REF/src/tokenizer.c $REF/src/parser.c $REF/src/parser/*.c $REF/src/utils.c $REF/src/csv_reader.c $REF/src/date_utils.c $REF/src/mmap.c"
FL="-O1 -g -w -fsanitize=address -fno-omit-frame-pointer -I$REF/include -Iinclude"
if [ "$2" = oracle ]; then
  gcc $FL -c oracle/cq_oracle.c -o $OUT/cq_oracle.o
  gcc $FL -o $OUT/asan_oracle scripts/asan_oracle.c $OUT/cq_oracle.o $SRC -lm
  ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 $OUT/asan_oracle "$1"
else
  gcc $FL -o $OUT/asan_parse scripts/asan_parse.c $SRC -lm
  ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0 $OUT/asan_parse "$1"
fi
