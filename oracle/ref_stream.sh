#!/bin/sh
# TEST INFRASTRUCTURE ONLY (oracle/_ref).  Writes to stdout, for gcc to read
# from a pipe, the listed line ranges of reference source files exactly as
# they are under $REF, each behind a `#line` directive naming its origin, after
# checking every range against the SHA-256 it had when the fixtures were made.
# Nothing is written to disk: `make ref` pipes this straight into the compiler.
#
#   ref_stream.sh <ref-root> <file> <first,last> <sha256> [<file> <range> <sha> ...]
set -e
root=$1
shift
while [ $# -ge 3 ]; do
    f=$1 range=$2 want=$3
    shift 3
    got=$(sed -n "${range}p" "$root/$f" | sha256sum | cut -d' ' -f1)
    if [ "$got" != "$want" ]; then
        # also into the pipe, so the compile fails whatever the shell does with the exit code
        echo "#error \"oracle/_ref: $f:$range is not the text the fixtures pin\""
        echo "oracle/_ref: $f:$range is not the text the fixtures pin ($got)" >&2
        exit 1
    fi
    printf '#line %s "%s"\n' "${range%%,*}" "$f"
    sed -n "${range}p" "$root/$f"
done
