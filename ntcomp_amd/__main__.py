import sys

from ntcomp_amd.cli import main

sys.exit(main())
