class UserUnavailableError(Exception):
    """The platform refused delivery because the user blocked / left the bot."""

    def __init__(self, chat_id=None, *args):
        super().__init__(chat_id, *args)
        self.chat_id = chat_id
