class UserUnavailableError(Exception):
    """The platform refused delivery because the user blocked / left the bot."""
