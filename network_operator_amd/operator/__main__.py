import sys

from .manager import main

sys.exit(main())
