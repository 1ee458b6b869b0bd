import sys

from midaspom_amd.cli import main

sys.exit(main())
