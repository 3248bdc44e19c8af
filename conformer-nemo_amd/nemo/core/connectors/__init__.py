from .save_restore_connector import SaveRestoreConnector, restore_modules  # noqa: F401
