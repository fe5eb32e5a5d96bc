# native apps are added in a later milestone
apps:
	@true
